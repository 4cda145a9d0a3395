"""Host-side frame loading (out of the accelerated scope)."""
