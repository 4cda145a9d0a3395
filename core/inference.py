"""Decode-policy registry (same names, values and fallback as the reference core/inference.py:4-16)."""
from __future__ import annotations

_PRESETS = {
    "precise": (3, 24, 1.0, 1.0, 3, 1.1),
    "detailed": (4, 40, 1.0, 1.0, 3, 1.1),
    "natural": (1, 24, 0.9, 0.9, 3, 1.05),
    "safe_sample": (1, 22, 0.8, 0.85, 3, 1.1),
}
_KEYS = ("num_beams", "max_new_tokens", "temperature", "top_p", "no_repeat_ngram_size", "repetition_penalty")


def preset_to_kwargs(name: str):
    """Decode policy registry for repeatable inference and benchmarking; unknown -> "precise"."""
    values = _PRESETS.get((name or "precise").lower(), _PRESETS["precise"])
    return dict(zip(_KEYS, values))
