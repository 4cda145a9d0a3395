"""frames_dir -> [1, T, 3, H, W] tensor (behaviour of reference core/preprocessing/frame_loader.py:13-49).

Strided pick files[::max(n // T, 1)][:T] of sorted frame_*.jpg.  For a cuda `device` the frames are
decoded on the GPU (vcap.jpeg: host entropy decode, device IDCT / upsampling / YCbCr -> RGB,
bit-identical to PIL's Image.open(...).convert("RGB")) and the Resize((S, S)) -> ToTensor ->
Normalize chain runs there too (vcap.preprocess, bit-identical to PIL's BILINEAR resample + the f32
normalisation).  `backend="pil"` keeps the per-frame host chain (PIL decode + resize + numpy), e.g.
for a CPU-only caller.  With `backend="auto"` on a cuda device, frames the GPU decoder refuses
(VCAP_E_UNSUPPORTED: progressive / arithmetic / RGB-coded JPEGs, frames of different sizes) are
decoded by PIL on the host, as the reference decodes every frame, and still resized and normalised
on the device; `backend="hip"` raises instead.  torchvision is not required.
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


def load_video_tensor(frames_dir, num_frames: int, image_size: int, device: str = "cuda",
                      backend: str = "auto") -> torch.Tensor:
    from PIL import Image
    files = list_frames(frames_dir)
    if not files:
        raise FileNotFoundError(f"No frame_*.jpg files found under {frames_dir}")
    picks = files[::max(len(files) // num_frames, 1)][:num_frames]
    on_gpu = torch.device(device).type == "cuda"
    strict = backend == "hip"   # an explicit GPU decode raises on what it refuses; "auto" falls back
    if backend == "auto":
        backend = "hip" if on_gpu else "pil"
    if backend not in ("hip", "pil"):
        raise ValueError(f"backend must be 'auto', 'hip' or 'pil', got {backend!r}")
    if on_gpu and backend == "hip":
        from vcap import _native as N
        from vcap.jpeg import decode_jpegs
        from vcap.preprocess import frames_to_video, preprocess_frames
        blobs = [Path(p).read_bytes() for p in picks]
        try:
            video = preprocess_frames(decode_jpegs(blobs, device), image_size).unsqueeze(0)
        except N.VcapError as e:
            if strict or e.rc != N.E_UNSUPPORTED:
                raise
            log.warning("GPU JPEG decode refused %s (%s): PIL host decode, device resize/normalise", frames_dir, e)
            pil = []
            for p in picks:
                with Image.open(p) as im:
                    pil.append(np.asarray(im.convert("RGB")))
            if any(a.shape != pil[0].shape for a in pil):
                video = torch.from_numpy(np.stack([_to_chw(Image.fromarray(a), image_size) for a in pil])[None]).to(device)
            else:
                video = frames_to_video(pil, image_size, device)
    elif backend == "hip":
        raise ValueError("backend='hip' needs a cuda device")
    else:
        decoded = []
        for p in picks:
            with Image.open(p) as im:
                decoded.append(_to_chw(im, image_size))
        video = torch.from_numpy(np.stack(decoded)[None]).to(device)
    log.info("frames_dir=%s total=%s sampled=%s", frames_dir, len(files), len(picks))
    return video
