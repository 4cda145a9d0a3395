"""Fused ViT token pool + temporal mean on the HIP path (replaces vit_fused_pool_temporal,
core/operators/cupy_vit_pool.py:127-186): returns None on unsupported shape/device, as the
reference does, so a caller can choose its own path; HIP errors raise."""
from __future__ import annotations

import torch

from vcap import _native as N


def vit_fused_pool_temporal(feat: torch.Tensor, bsz: int, timesteps: int, pool: str, force_bf16: bool = False):
    if not feat.is_cuda or feat.ndim != 3 or pool not in {"cls", "gap"}:
        return None
    bt, tokens, channels = feat.shape
    if bt != bsz * timesteps or (pool == "gap" and tokens <= 1):
        return None
    dt, tdt = (N.DT_BF16, torch.bfloat16) if (force_bf16 or feat.dtype == torch.bfloat16) else (N.DT_F32, torch.float32)
    x = feat.to(tdt).contiguous()
    out = torch.empty(bsz, channels, dtype=tdt, device=feat.device)
    N.check(N.lib().vcap_vit_pool_temporal(dt, x.data_ptr(), out.data_ptr(), bsz, timesteps, tokens, channels,
                                           int(pool == "gap"), torch.cuda.current_stream(feat.device).cuda_stream),
            "vcap_vit_pool_temporal")
    return out
