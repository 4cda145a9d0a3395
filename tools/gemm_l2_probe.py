"""Is the 256x256 GEMM K-loop waiting on memory?  The ViT fc1 / fc2 shapes (25216 rows) through
vcap_gemm (policy 2) with the operands as they are, and with overlapping rows (row stride 64
elements: the A rows, or A and W, then span a few MB that stay in L2), same tile count and
instruction stream.  Prints us per launch (median of 5 rounds of 10 launches)."""
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402

M = 25216
dev = torch.device("cuda:0")
lib = N.lib()
N.check(lib.vcap_set_gemm_policy(2), "policy")
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device=dev).manual_seed(0)


def rnd(n, scale=1.0):
    return ((torch.rand(n, generator=g, device=dev) * 2 - 1) * scale).bfloat16()


shapes = {"fc1": (3072, 768, False, 1), "fc2": (768, 3072, True, 0), "qkv": (2304, 768, False, 0)}
for name, (n, k, f32, act) in shapes.items():
    b = (torch.rand(n, generator=g, device=dev) * 0.2 - 0.1)
    C = torch.zeros(M, n, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
    odt = N.DT_F32 if f32 else N.DT_BF16
    A_full, W_full = rnd(M * k), rnd(n * k, 0.05)
    A_alias, W_alias = rnd(M * 64 + k), rnd(n * 64 + k, 0.05)
    variants = {"as is": (A_full, k, W_full, k), "A rows overlap": (A_alias, 64, W_full, k),
                "A+W rows overlap": (A_alias, 64, W_alias, 64)}
    res = {v: [] for v in variants}

    def run(v, reps):
        A, lda, W, ldw = variants[v]
        for _ in range(reps):
            N.check(lib.vcap_gemm(N.DT_BF16, odt, A.data_ptr(), lda, W.data_ptr(), ldw, C.data_ptr(), n, M, n, k,
                                  b.data_ptr(), act, C.data_ptr() if f32 else None, n if f32 else 0, 1 if f32 else 0,
                                  0, 0, 0, 0, s), name)

    for v in variants:
        run(v, 3)
    for _ in range(5):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(v, 10)
            e1.record()
            e1.synchronize()
            res[v].append(e0.elapsed_time(e1) / 10 * 1e3)
    fl = 2.0 * M * n * k
    print(f"{name} M={M} N={n} K={k}: " + "  ".join(
        f"{v}: {statistics.median(t):6.1f} us ({fl / statistics.median(t) / 1e6:5.0f} TF/s)" for v, t in res.items()),
        flush=True)
