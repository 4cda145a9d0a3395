"""Decoded RGB frames -> the encoder's normalised input on the GPU (vcap_frames_preprocess).

Replaces the per-frame host transform chain of core/preprocessing/frame_loader.py:34-45
(torchvision Resize((S, S)) -> ToTensor -> Normalize) with one upload of the uint8 frames and three
kernels (weights, horizontal pass, vertical pass + normalise), bit-identical to PIL's BILINEAR
resample and the reference's f32 normalisation.  The JPEG decode in front of it is vcap.jpeg (also on
the GPU).  There is no host fallback: a missing libvcap_hip.so raises.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np
import torch

from . import _native as N

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def preprocess_frames(frames_u8: torch.Tensor, size: int, mean: Sequence[float] = IMAGENET_MEAN,
                      std: Sequence[float] = IMAGENET_STD, out_u8: bool = False):
    """frames_u8 [n, H, W, 3] uint8 (device) -> [n, 3, size, size] f32 (and the resized uint8 pixels
    [n, size, size, 3] when out_u8)."""
    if frames_u8.dim() != 4 or frames_u8.shape[-1] != 3 or frames_u8.dtype != torch.uint8 or not frames_u8.is_cuda:
        raise ValueError(f"expect a cuda uint8 [n, H, W, 3] tensor, got {frames_u8.dtype} {tuple(frames_u8.shape)}")
    x = frames_u8.contiguous()
    n, h, w, _ = x.shape
    lib = N.lib()
    out = torch.empty(n, 3, size, size, dtype=torch.float32, device=x.device)
    u8 = torch.empty(n, size, size, 3, dtype=torch.uint8, device=x.device) if out_u8 else None
    ws = torch.empty(max(int(lib.vcap_frames_workspace_bytes(n, h, w, size, size)), 1), dtype=torch.uint8,
                     device=x.device)
    m = (C.c_float * 3)(*mean)
    sd = (C.c_float * 3)(*std)
    N.check(lib.vcap_frames_preprocess(x.data_ptr(), n, h, w, size, size, m, sd, out.data_ptr(), N.ptr(u8),
                                       ws.data_ptr(), ws.numel(), torch.cuda.current_stream(x.device).cuda_stream),
            "vcap_frames_preprocess")
    return (out, u8) if out_u8 else out


def frames_to_video(frames: Sequence[np.ndarray], size: int, device) -> torch.Tensor:
    """Decoded RGB frames (host uint8 [H, W, 3], one size) -> video [1, T, 3, size, size] on device."""
    arr = np.stack([np.asarray(f, dtype=np.uint8) for f in frames])
    x = torch.from_numpy(arr).to(device)
    return preprocess_frames(x, size).unsqueeze(0)
