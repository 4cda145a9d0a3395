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


def jpeg_cases():
    """Generated JPEG test images: (name, bytes).  Smooth colour fields plus noise (real AC content),
    every chroma subsampling Pillow writes (4:4:4, 4:2:2, 4:2:0), qualities 50 / 95 / 100 (quantiser
    1 everywhere at 100: full-range coefficients), odd sizes (partial MCUs, odd chroma widths),
    greyscale, and restart intervals."""
    import io

    from PIL import Image
    rs = np.random.RandomState(0)

    def img(h, w, mode="RGB"):
        yy, xx = np.mgrid[0:h, 0:w]
        base = np.stack([128 + 100 * np.sin(xx / 7.0 + c) * np.cos(yy / 5.0 - c) for c in range(3)], -1)
        a = np.clip(base + rs.randn(h, w, 3) * 30, 0, 255).astype(np.uint8)
        im = Image.fromarray(a)
        return im.convert("L") if mode == "L" else im

    out = []
    specs = [((h, w), ss, q, "RGB", {}) for (h, w) in [(37, 53), (64, 48), (17, 9), (120, 160)]
             for ss in (0, 1, 2) for q in (50, 95, 100)]
    specs += [((37, 53), None, 90, "L", {}), ((64, 80), 2, 85, "RGB", {"restart_marker_blocks": 3}),
              ((64, 80), 2, 85, "RGB", {"restart_marker_rows": 1}), ((240, 320), 2, 90, "RGB", {})]
    for (h, w), ss, q, mode, kw in specs:
        b = io.BytesIO()
        kws = dict(format="JPEG", quality=q, **kw)
        if ss is not None:
            kws["subsampling"] = ss
        img(h, w, mode).save(b, **kws)
        out.append((f"{h}x{w}_{mode}_ss{ss}_q{q}{'_' + '_'.join(kw) if kw else ''}", b.getvalue()))
    return out
