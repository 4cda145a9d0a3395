"""nn.Linear drop-in on the HIP path (replaces CuPyLinearCompat, core/operators/cupy_linear_mapper.py:137-184).

Same parameter names (weight/bias) for checkpoint compatibility and the same bookkeeping
attributes (`last_backend`, `last_error`).  CUDA inputs run vcap_linear_bias (fp32, or bf16 with
fp32 accumulation when force_bf16); a failing HIP call raises (strict=True, the default) instead
of silently falling back, and so does a CPU input.  torch's Linear runs only when asked for:
enabled=False, strict=False, or autograd (training / requires_grad - the HIP op has no backward,
and training is outside this path).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from vcap import _native as N


class HipLinearCompat(nn.Linear):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, enabled: bool = True,
                 force_bf16: bool = False, strict: bool = True):
        super().__init__(in_features, out_features, bias=bias)
        self.enabled, self.force_bf16, self.strict = enabled, force_bf16, strict
        self.last_backend, self.last_error = "torch", ""

    def _use_hip(self, x: torch.Tensor) -> bool:
        return self.enabled and x.is_cuda and not self.training and not x.requires_grad

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.enabled and self.strict and not x.is_cuda and not (self.training or x.requires_grad):
            raise RuntimeError("HipLinearCompat: the HIP path needs a GPU tensor (strict=True); "
                               "use enabled=False or strict=False for torch's Linear")
        if not self._use_hip(x):
            self.last_backend, self.last_error = "torch", ""
            return super().forward(x)
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        dt, tdt = (N.DT_BF16, torch.bfloat16) if (self.force_bf16 or x.dtype == torch.bfloat16) else (N.DT_F32, torch.float32)
        xw = x2.to(tdt).contiguous()
        w = self.weight.detach().to(tdt).contiguous()
        b = self.bias.detach().float().contiguous() if self.bias is not None else None
        y = torch.empty(xw.shape[0], self.out_features, dtype=tdt, device=x.device)
        try:
            N.check(N.lib().vcap_linear_bias(dt, xw.data_ptr(), w.data_ptr(), N.ptr(b), y.data_ptr(), xw.shape[0],
                                             self.in_features, self.out_features,
                                             torch.cuda.current_stream(x.device).cuda_stream), "vcap_linear_bias")
        except Exception as exc:  # noqa: BLE001
            self.last_backend, self.last_error = "hip_error", str(exc)
            raise
        self.last_backend, self.last_error = "hip", ""
        return y.reshape(*shape[:-1], self.out_features)
