"""Shared fixtures-as-functions for the parity tests (seeded weights/frames + golden loading)."""
from __future__ import annotations

import json
from functools import lru_cache
from pathlib import Path

import numpy as np

from vcap import configs, prng, weights

GOLDEN = Path(__file__).resolve().parent / "golden"


@lru_cache(maxsize=None)
def golden(name: str):
    meta = json.loads((GOLDEN / f"{name}.json").read_text())
    arrays = dict(np.load(GOLDEN / f"{name}.npz"))
    return meta, arrays


@lru_cache(maxsize=4)
def state_dict(vit: str, gpt2: str, seed: int):
    return weights.synthetic_state_dict(seed, configs.vit_arch(vit), configs.gpt2_arch(gpt2))


def case(name: str):
    """(meta, arrays, vit_arch, gpt2_arch, state_dict, frames[B,T,3,H,W] np.float32)."""
    meta, arrays = golden(name)
    va, ga = configs.vit_arch(meta["vit"]), configs.gpt2_arch(meta["gpt2"])
    sd = state_dict(meta["vit"], meta["gpt2"], meta["weights_seed"])
    frames = prng.imagenet_frames(meta["frames_seed"], (meta["B"], meta["T"], 3, va.image, va.image))
    return meta, arrays, va, ga, sd, frames


def pad_rows(rows, width, fill=-1):
    out = np.full((len(rows), width), fill, np.int32)
    for i, r in enumerate(rows):
        out[i, :len(r)] = r
    return out
