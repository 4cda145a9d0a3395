"""256x256 kernel (policy 2) vs 128x128 (policy 1) on square / long-K shapes, random bf16 data:
separates the K-loop rate from per-tile prologue/epilogue and last-round quantisation."""
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402

dev = torch.device("cuda:0")
lib = N.lib()
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device=dev).manual_seed(0)
for (M, n, k) in [(4096, 4096, 4096), (8192, 8192, 8192), (25216, 3072, 768), (25216, 3072, 6144),
                  (16384, 4096, 768), (8192, 4096, 768)]:
    A = (torch.rand(M, k, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand(n, k, generator=g, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
    C = torch.empty(M, n, device=dev, dtype=torch.bfloat16)
    row = [f"M={M} N={n} K={k}:"]
    for p in (1, 2):
        lib.vcap_set_gemm_policy(p)
        for _ in range(3):
            lib.vcap_gemm(N.DT_BF16, N.DT_BF16, A.data_ptr(), k, W.data_ptr(), k, C.data_ptr(), n, M, n, k,
                          None, 0, None, 0, 0, 0, 0, 0, 0, s)
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                lib.vcap_gemm(N.DT_BF16, N.DT_BF16, A.data_ptr(), k, W.data_ptr(), k, C.data_ptr(), n, M, n, k,
                              None, 0, None, 0, 0, 0, 0, 0, 0, s)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 5)
        ms = statistics.median(ts)
        row.append(f"tile{128 if p == 1 else 256} {ms * 1e3:8.1f} us {2.0 * M * n * k / ms / 1e9:7.1f} TF")
    print("  ".join(row), flush=True)
    del A, W, C
lib.vcap_set_gemm_policy(0)
