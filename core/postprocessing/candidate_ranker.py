"""Heuristic candidate scoring (behaviour of the reference core/postprocessing/candidate_ranker.py:7-36),
written as a rule table; pinned by tests/golden/text_rules.json produced from the reference itself."""
from __future__ import annotations

import re
from typing import Iterable, Tuple

_MU, _SIGMA = 12.0, 4.0
# (predicate on the text, score delta)
_RULES = (
    (lambda t: re.search(r"\b\w+ing\b", t) is not None, 1.0),
    (lambda t: re.search(r"\b(?:is|are|was|were)\b", t) is not None, 0.5),
    (lambda t: t.endswith((".", "!", "?")), 0.3),
    (lambda t: re.search(r"\b(?:[A-Z]\.){2,}\b", t) is not None, -1.5),
    (lambda t: re.search(r"(?i)\b(click here|subscribe|report abuse|sign up|pastebin)\b", t) is not None, -1.5),
    (lambda t: len(t.split()) < 4, -2.0),
    (lambda t: t.strip().lower() in {"someone is sitting.", "someone is in the scene."}, -0.8),
)


def score_sentence(text: str) -> float:
    if not text:
        return -1e9
    n = len(text.split())
    return -((n - _MU) ** 2) / (2 * _SIGMA * _SIGMA) + sum(delta for pred, delta in _RULES if pred(text))


def select_best(candidates: Iterable[Tuple[str, str]]):
    """Highest score wins; the first candidate wins ties (stable sort order of the reference)."""
    best = None
    for key, value in candidates:
        s = score_sentence(value)
        if best is None or s > best[2]:
            best = (key, value, s)
    return best
