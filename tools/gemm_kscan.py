"""Per-launch time of the 256x256 GEMM (policy 2) at M=25216 over K, for bf16-out (QKV/fc1 epilogue)
and f32-out + residual (attn-proj/fc2 epilogue) at N = 3072 / 768.  The intercept of time vs K is
the per-tile fixed cost (pipeline fill + epilogue); the slope is the K-loop rate."""
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 25216
dev = torch.device("cuda:0")
lib = N.lib()
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device=dev).manual_seed(0)
N.check(lib.vcap_set_gemm_policy(int(sys.argv[2]) if len(sys.argv) > 2 else 2), "policy")


def rnd(*shape, scale=1.0, dtype=torch.bfloat16):
    return (torch.rand(*shape, generator=g, device=dev) * 2 - 1).mul_(scale).to(dtype)


for n, f32 in ((3072, False), (2304, False), (768, True)):
    for k in (256, 512, 768, 1536, 3072):
        A, W = rnd(M, k), rnd(n, k, scale=0.05)
        b = rnd(n, scale=0.1, dtype=torch.float32)
        C = torch.zeros(M, n, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        odt = N.DT_F32 if f32 else N.DT_BF16

        def run(reps):
            for _ in range(reps):
                N.check(lib.vcap_gemm(N.DT_BF16, odt, A.data_ptr(), k, W.data_ptr(), k, C.data_ptr(), n, M, n, k,
                                      b.data_ptr(), 0, C.data_ptr() if f32 else None, n if f32 else 0,
                                      1 if f32 else 0, 0, 0, 0, 0, s), "gemm")
        run(3)
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(10)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        ms = statistics.median(ts)
        print(f"N={n:5d} K={k:5d} {'f32+res' if f32 else 'bf16   '} {ms * 1e3:8.1f} us "
              f"{2.0 * M * n * k / ms / 1e9:7.1f} TF", flush=True)
