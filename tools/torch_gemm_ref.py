"""Calibration: the same ViT GEMM shapes through torch (hipBLASLt) - plain bf16 Linear with bias,
no fused GELU / residual - next to nothing else.  Prints us and TFLOP/s per shape."""
import statistics
import torch
import torch.nn.functional as F

M = 25216
dev = torch.device("cuda:0")
for name, n, k in (("qkv", 2304, 768), ("proj", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072)):
    a = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.05
    b = torch.randn(n, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        F.linear(a, w, b)
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            F.linear(a, w, b)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    ms = statistics.median(ts)
    print(f"{name:5s} M={M} N={n} K={k}: torch/hipBLASLt {ms * 1e3:7.1f} us {2 * M * n * k / ms / 1e9:7.1f} TF", flush=True)
