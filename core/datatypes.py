"""Result types of the engine surface (reference core/datatypes.py:7-30)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict


@dataclass(frozen=True)
class CaptionCandidates:
    s1: str
    s2: str
    s3: str


@dataclass(frozen=True)
class InferenceResult:
    candidates: CaptionCandidates
    best_key: str
    best_text: str

    def to_api_dict(self) -> Dict[str, object]:
        c = self.candidates
        return {"S1": c.s1, "S2": c.s2, "S3": c.s3, "BEST": {"key": self.best_key, "text": self.best_text}}
