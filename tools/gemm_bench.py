"""ViT GEMM shapes (B=8 videos x 16 frames x 197 tokens = 25216 rows, ViT-B/16) through vcap_gemm
with the 128x128 kernel (policy 1) and the 256x256 8-phase kernel (policy 2), interleaved rounds in
one process on random bf16 operands.  Prints TFLOP/s per shape and policy (median of rounds)."""
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


def rnd(*shape, scale=1.0, dtype=torch.bfloat16):
    return (torch.rand(*shape, generator=g, device=dev) * 2 - 1).mul_(scale).to(dtype)


shapes = {  # name: (N, K, out f32?, act, residual)
    "qkv": (2304, 768, False, 0, False),
    "proj": (768, 768, True, 0, True),
    "fc1": (3072, 768, False, 1, False),
    "fc2": (768, 3072, True, 0, True),
}
bufs = {}
for name, (n, k, f32, act, res) in shapes.items():
    A = rnd(M, k)
    W = rnd(n, k, scale=0.05)
    b = rnd(n, scale=0.1, dtype=torch.float32)
    C = torch.zeros(M, n, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
    bufs[name] = (A, W, b, C)


def run(name, reps):
    n, k, f32, act, res = shapes[name]
    A, W, b, C = bufs[name]
    odt = N.DT_F32 if f32 else N.DT_BF16
    for _ in range(reps):
        N.check(lib.vcap_gemm(N.DT_BF16, odt, A.data_ptr(), k, W.data_ptr(), k, C.data_ptr(), n, M, n, k,
                              b.data_ptr(), act, C.data_ptr() if res else None, n if res else 0, 1 if res else 0,
                              0, 0, 0, 0, s), name)


POL = (1, 2, 0)
times = {(nm, p): [] for nm in shapes for p in POL}
for p in POL:
    lib.vcap_set_gemm_policy(p)
    for nm in shapes:
        run(nm, 3)
torch.cuda.synchronize()
for rnd_i in range(5):
    for p in POL:
        lib.vcap_set_gemm_policy(p)
        for nm in shapes:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(nm, 10)
            e1.record()
            e1.synchronize()
            times[(nm, p)].append(e0.elapsed_time(e1) / 10)
lib.vcap_set_gemm_policy(0)
for nm, (n, k, *_) in shapes.items():
    fl = 2.0 * M * n * k
    row = [f"{nm:5s} M={M} N={n} K={k}:"]
    for p in POL:
        ms = statistics.median(times[(nm, p)])
        row.append(f"{['auto', 'tile128', 'tile256'][p]} {ms * 1e3:7.1f} us {fl / ms / 1e9:7.1f} TF")
    print("  ".join(row), flush=True)
