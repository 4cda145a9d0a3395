"""Caption clean-up (behaviour of the reference core/postprocessing/text_cleaner.py:77-122).

Expressed as an ordered pipeline of stages; pinned by tests/golden/text_rules.json, which records
the reference's own clean_text() outputs for a corpus of inputs."""
from __future__ import annotations

import re

from core.postprocessing.candidate_ranker import score_sentence

_SPACES = re.compile(r"\s{2,}")
_REJECT_FULL = (re.compile(r"[-_= \t]{6,}\.?"), re.compile(r'"\s*[^"]+\s*"\.?'))
_REJECT_HEAD = re.compile(r"^\s*(https?://|www\.|<a\b|&lt;a\b)|^\s*(copyright\b)", re.I)
_BAD_LEADS = re.compile(r"^\s*(?:" + "|".join((
    r"you are about to\b", r"click here\b", r"subscribe\b", r"available on youtube\b", r"watch live\b",
    r"find out\b", r"the video will\b", r"on the road\b")) + r")", re.I)
_REJECT_ANY = re.compile(r"(</?\w+>|reddit\.com|pastebin|mailto:)", re.I)
_SPAM = r"(?i)\b(click here|subscribe|report abuse|pastebin|official facebook|video will be"
_COUNTRY_RULES = ((r"\bU\.S\.A?\.?\b", re.I), (r"\bUSA\b", re.I), (r"\bUnited States of America\b", re.I),
                  (r"\bUnited States\b", re.I), (r"\bAmerica\b", re.I))
_PREP_RULES = ((r"(?i)\bin\s+the\s+front\s+of\b", "in front of"), (r"(?i)\bin\s+the\s+middle\s+of\b", "in the middle of"),
               (r"(?i)\bat\s+the\s+side\s+of\b", "at the side of"))


def _squash(t: str) -> str:
    return _SPACES.sub(" ", t)


def _drop_countries(t: str) -> str:
    for pat, fl in _COUNTRY_RULES:
        t = re.sub(pat, "", t, flags=fl)
    return _squash(t).strip()


def _prep_chains(t: str) -> str:
    for pat, rep in _PREP_RULES:
        t = re.sub(pat, rep, t)
    return _squash(t)


def _noise_cut_index(tokens) -> int:
    for i, tok in enumerate(tokens):
        core = tok.strip(",.;:!?()[]{}\"'`")
        if not core:
            continue
        if (re.search(r"[0-9/\\]", core) or re.match(r"^(?:[A-Za-z]\.){2,}$", core)
                or re.match(r"^[A-Z]{1,3}-[A-Za-z0-9]{1,6}$", core) or (len(core) <= 3 and core.isupper())):
            return i
    return len(tokens)


def _truncate_noise(t: str) -> str:
    if not t:
        return t
    toks = t.split()
    out = " ".join(toks[:_noise_cut_index(toks)]).strip()
    return out + "." if out and out[-1] not in ".!?" else out


def _prune_tails(t: str) -> str:
    t = re.sub(r"(?i)\b(?:how|why|what|that|which)\b.*$", "", t).strip()
    t = re.sub(r"(?i)\bA\s+wonders\b.*$", "", t).strip()
    return t or "Someone is in the scene."


def _sit_complement(t: str) -> str:
    low = t.strip().lower()
    if re.match(r"^someone\s+is\b", low):
        return t  # the reference returns early here, so the two sitting rules below never fire
    if re.match(r"^someone\s+is\s+sitting\s*\.?$", low):
        return "Someone is sitting on a chair."
    if re.match(r"^someone\s+is\s+sitting\b", low) and not re.search(r"\b(in|on|at|by|with|near)\b", low):
        return t.rstrip(". ") + " on a chair."
    return t


def _caps_period(t: str) -> str:
    t = t.strip()
    if t and t[0].isalpha():
        t = t[0].upper() + t[1:]
    return t + "." if t and t[-1] not in ".!?" else t


def clean_text(raw: str) -> str:
    t = (raw or "").strip()
    if _REJECT_FULL[0].fullmatch(t):
        return ""
    t = re.sub(r"^\s*[-_= \t]{2,}\s*", "", t)
    if _REJECT_HEAD.match(t) or _REJECT_FULL[1].fullmatch(t) or _BAD_LEADS.match(t) or _REJECT_ANY.search(t):
        return ""
    spam = re.search(_SPAM + r")\b", t) is not None
    t = re.sub(_SPAM + r".*)$", "", t).strip()
    t = _prep_chains(_drop_countries(t))
    if len(t.split()) >= 10:
        t = _truncate_noise(t)
    t = _prune_tails(t)
    if spam and len(t.split()) <= 2:
        t = "Someone is in the scene."
    t = _sit_complement(t)
    t = re.sub(r"(?i)\b(\w+)\b(?:\s+\1\b)+", r"\1", t)
    t = _caps_period(_squash(t).strip())
    parts = [p.strip() for p in re.split(r"\s*(?<=\.|\!|\?)\s+", t) if p.strip()]
    if len(parts) > 1:
        t = max(parts, key=score_sentence)
    return parts[0] if parts and parts[0] else t
