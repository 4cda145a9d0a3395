"""Interleaved A/B timing of the ViT GEMM shapes across library builds / GEMM policies in ONE
process (box-to-box clock differences cancel).  usage: gemm_ab.py [M] lib.so:policy ...
('-' as the library = the in-tree build)."""
import ctypes as C
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
M = int(args.pop(0)) if args and args[0].isdigit() else 25216
variants = []
for a in args:
    path, pol = a.rsplit(":", 1)
    h = C.CDLL(str(N.library_path()) if path == "-" else path, mode=C.RTLD_LOCAL)
    for name in ("vcap_gemm", "vcap_set_gemm_policy", "vcap_last_error"):
        res, at = N.SIGNATURES[name]
        getattr(h, name).restype, getattr(h, name).argtypes = res, at
    variants.append((a, h, int(pol)))

dev = torch.device("cuda:0")
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*shape, scale=1.0, dtype=torch.bfloat16):
    return (torch.rand(*shape, generator=g, device=dev) * 2 - 1).mul_(scale).to(dtype)


shapes = {"qkv": (2304, 768, False, 0), "proj": (768, 768, True, 0), "fc1": (3072, 768, False, 1),
          "fc2": (768, 3072, True, 0)}
if "--with-nogelu" in sys.argv:
    shapes["fc1_nogelu"] = (3072, 768, False, 0)
bufs = {}
for name, (n, k, f32, act) in shapes.items():
    bufs[name] = (rnd(M, k), rnd(n, k, scale=0.05), rnd(n, scale=0.1, dtype=torch.float32),
                  torch.zeros(M, n, device=dev, dtype=torch.float32 if f32 else torch.bfloat16))


def run(h, name, reps):
    n, k, f32, act = shapes[name]
    A, W, b, Cc = bufs[name]
    for _ in range(reps):
        rc = h.vcap_gemm(N.DT_BF16, N.DT_F32 if f32 else N.DT_BF16, A.data_ptr(), k, W.data_ptr(), k, Cc.data_ptr(),
                         n, M, n, k, b.data_ptr(), act, Cc.data_ptr() if f32 else None, n if f32 else 0,
                         1 if f32 else 0, 0, 0, 0, 0, s)
        if rc:
            raise RuntimeError(f"{name}: {h.vcap_last_error()}")


ref = {}
for tag, h, pol in variants:
    assert h.vcap_set_gemm_policy(pol) == 0
    for nm in shapes:
        run(h, nm, 2)
        torch.cuda.synchronize()
        ref.setdefault(nm, bufs[nm][3].clone())
        bufs[nm][3].zero_()
times = {(tag, nm): [] for tag, _, _ in variants for nm in shapes}
for _ in range(7):
    for tag, h, pol in variants:
        h.vcap_set_gemm_policy(pol)
        for nm in shapes:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(h, nm, 10)
            e1.record()
            e1.synchronize()
            times[(tag, nm)].append(e0.elapsed_time(e1) / 10)
for nm, (n, k, *_) in shapes.items():
    fl = 2.0 * M * n * k
    row = [f"{nm:5s} N={n} K={k}:"]
    for tag, _, _ in variants:
        ms = statistics.median(times[(tag, nm)])
        row.append(f"{tag.split('/')[-1]} {ms * 1e3:7.1f} us {fl / ms / 1e9:6.0f} TF")
    print("  ".join(row), flush=True)
