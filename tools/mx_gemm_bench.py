"""MXFP8 vs bf16 256x256 GEMM throughput at the ViT shapes (M = 25216 rows: 8 videos x 16 frames x
197 tokens) and square shapes.  Prints TFLOP/s (median of 20 launches, HIP events on the launch
stream) per shape: bf16 (vcap_gemm, policy 2) and MXFP8 (vcap_gemm_mx)."""
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402

dev = torch.device("cuda:0")
lib = N.lib()
N.check(lib.vcap_set_gemm_policy(2), "policy")
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device=dev).manual_seed(0)


def quant(x):
    rows, K = x.shape
    q = torch.empty(rows, K, dtype=torch.uint8, device=dev)
    sc = torch.empty(int(lib.vcap_mx_scale_bytes(rows, K)), dtype=torch.uint8, device=dev)
    N.check(lib.vcap_mx_quantize(N.DT_F32, x.data_ptr(), K, rows, K, q.data_ptr(), sc.data_ptr(), s), "q")
    return q, sc


def timed(fn, reps=20):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


import os  # noqa: E402
MR = int(os.environ.get("M_ROWS", "25216"))   # 50432 = the 16-video encode of the fp8 bench line
shapes = [("qkv", MR, 2304, 768, "bf16", 0), ("fc1", MR, 3072, 768, "fp8", 1),
          ("fc2", MR, 768, 3072, "f32", 0), ("sq4096", 4096, 4096, 4096, "bf16", 0),
          ("sq8192", 8192, 8192, 8192, "bf16", 0)]
for name, M, Nn, K, out, act in shapes:
    A = torch.rand(M, K, generator=g, device=dev) * 2 - 1
    W = (torch.rand(Nn, K, generator=g, device=dev) * 2 - 1) * 0.05
    bias = torch.zeros(Nn, device=dev)
    Ab, Wb = A.bfloat16(), W.bfloat16()
    Cb = torch.empty(M, Nn, device=dev, dtype=torch.float32 if out == "f32" else torch.bfloat16)
    fl = 2.0 * M * Nn * K
    tb = timed(lambda: N.check(lib.vcap_gemm(N.DT_BF16, N.DT_F32 if out == "f32" else N.DT_BF16, Ab.data_ptr(), K,
                                             Wb.data_ptr(), K, Cb.data_ptr(), Nn, M, Nn, K, bias.data_ptr(),
                                             act if out != "f32" else 0, None, 0, 0, 0, 0, 0, 0, s), "bf16"))
    aq, asc = quant(A)
    wq, wsc = quant(W)
    odt = {"bf16": N.DT_BF16, "f32": N.DT_F32, "fp8": N.DT_MXFP8}[out]
    Cq = torch.empty(M, Nn, device=dev, dtype={"bf16": torch.bfloat16, "f32": torch.float32, "fp8": torch.uint8}[out])
    csc = torch.empty(int(lib.vcap_mx_scale_bytes(M, Nn)), dtype=torch.uint8, device=dev)
    tq = timed(lambda: N.check(lib.vcap_gemm_mx(aq.data_ptr(), asc.data_ptr(), wq.data_ptr(), wsc.data_ptr(), odt,
                                                Cq.data_ptr(), Nn, csc.data_ptr() if out == "fp8" else None, M, Nn, K,
                                                bias.data_ptr(), act, None, s), "mx"))
    print(f"{name:7s} M={M} N={Nn} K={K}: bf16 {tb * 1e3:8.1f} us {fl / tb / 1e9:7.1f} TF/s | "
          f"mxfp8 {tq * 1e3:8.1f} us {fl / tq / 1e9:7.1f} TF/s", flush=True)

# VARIANTS=1: the fc1 shape with each epilogue, to split the MXFP8 fc1 launch's cost between the
# K loop and its bias + GELU + MXFP8-requantising epilogue (EPI 4)
if os.environ.get("VARIANTS"):
    M, Nn, K = MR, 3072, 768
    A = torch.rand(M, K, generator=g, device=dev) * 2 - 1
    W = (torch.rand(Nn, K, generator=g, device=dev) * 2 - 1) * 0.05
    bias = torch.zeros(Nn, device=dev)
    aq, asc = quant(A)
    wq, wsc = quant(W)
    Ab, Wb = A.bfloat16(), W.bfloat16()
    fl = 2.0 * M * Nn * K
    Cb = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    Cq = torch.empty(M, Nn, device=dev, dtype=torch.uint8)
    csc = torch.empty(int(lib.vcap_mx_scale_bytes(M, Nn)), dtype=torch.uint8, device=dev)
    for label, fn in [
        ("bf16 in, bf16 out", lambda: lib.vcap_gemm(N.DT_BF16, N.DT_BF16, Ab.data_ptr(), K, Wb.data_ptr(), K, Cb.data_ptr(),
                                                     Nn, M, Nn, K, bias.data_ptr(), 0, None, 0, 0, 0, 0, 0, 0, s)),
        ("bf16 in, bf16 GELU out", lambda: lib.vcap_gemm(N.DT_BF16, N.DT_BF16, Ab.data_ptr(), K, Wb.data_ptr(), K,
                                                          Cb.data_ptr(), Nn, M, Nn, K, bias.data_ptr(), 1, None, 0, 0, 0,
                                                          0, 0, 0, s)),
        ("mx in, bf16 out", lambda: lib.vcap_gemm_mx(aq.data_ptr(), asc.data_ptr(), wq.data_ptr(), wsc.data_ptr(),
                                                      N.DT_BF16, Cb.data_ptr(), Nn, None, M, Nn, K, bias.data_ptr(), 0,
                                                      None, s)),
        ("mx in, bf16 GELU out", lambda: lib.vcap_gemm_mx(aq.data_ptr(), asc.data_ptr(), wq.data_ptr(), wsc.data_ptr(),
                                                           N.DT_BF16, Cb.data_ptr(), Nn, None, M, Nn, K, bias.data_ptr(),
                                                           1, None, s)),
        ("mx in, mx GELU out", lambda: lib.vcap_gemm_mx(aq.data_ptr(), asc.data_ptr(), wq.data_ptr(), wsc.data_ptr(),
                                                         N.DT_MXFP8, Cq.data_ptr(), Nn, csc.data_ptr(), M, Nn, K,
                                                         bias.data_ptr(), 1, None, s)),
    ]:
        t = timed(lambda: N.check(fn(), label))
        print(f"fc1 shape M={M} {label:24s} {t * 1e3:8.1f} us {fl / t / 1e9:7.1f} TF/s", flush=True)
