"""frames_dir -> [1, T, 3, H, W] tensor (behaviour of reference core/preprocessing/frame_loader.py:13-49).

Strided pick files[::max(n // T, 1)][:T] of sorted frame_*.jpg, PIL bilinear resize to (H, W)
(what torchvision Resize does for PIL images), /255, ImageNet mean/std normalisation.  torchvision
is not required.  Frames are uploaded once; the HIP encoder consumes them from HBM.
"""
from __future__ import annotations

import logging
from pathlib import Path

import numpy as np
import torch

log = logging.getLogger(__name__)
_MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
_STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def list_frames(frames_dir: Path):
    return sorted(Path(frames_dir).glob("frame_*.jpg"))


def _to_chw(img, size: int) -> np.ndarray:
    from PIL import Image
    img = img.convert("RGB").resize((size, size), Image.BILINEAR)
    arr = np.asarray(img, dtype=np.float32) / 255.0
    return ((arr - _MEAN) / _STD).transpose(2, 0, 1)


def load_video_tensor(frames_dir, num_frames: int, image_size: int, device: str = "cuda") -> torch.Tensor:
    from PIL import Image
    files = list_frames(frames_dir)
    if not files:
        raise FileNotFoundError(f"No frame_*.jpg files found under {frames_dir}")
    picks = files[::max(len(files) // num_frames, 1)][:num_frames]
    frames = []
    for p in picks:
        with Image.open(p) as im:
            frames.append(_to_chw(im, image_size))
    video = torch.from_numpy(np.stack(frames)[None]).to(device)
    log.info("frames_dir=%s total=%s sampled=%s", frames_dir, len(files), len(picks))
    return video
