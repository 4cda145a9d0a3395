"""Prefix normalisation op (reference core/operators/normalization.py:6-13 semantics).  On CUDA
tensors the HIP engine path fuses it with the mapper (vcap_prefix_project); this helper is the
plain tensor form for callers that hold an embedding."""
from __future__ import annotations

import torch


def apply_prefix_norm(prefix: torch.Tensor, ln_scale: float, in_weight: float) -> torch.Tensor:
    if ln_scale is not None and ln_scale > 0:
        prefix = torch.nn.functional.layer_norm(prefix, prefix.shape[-1:]) * ln_scale
    if in_weight is not None and in_weight > 0:
        prefix = prefix * in_weight
    return prefix
