"""Host-side caption post-processing (out of the accelerated scope; kept so infer() output matches)."""
