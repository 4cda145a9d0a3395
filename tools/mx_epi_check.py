"""Dump the MXFP8 fc1-shape GEMM output (bias + GELU -> MXFP8 bytes + E8M0 scales) of the library named
by VCAP_LIB to <out>.npz, or compare two dumps bit for bit: an epilogue store-layout variant must
produce identical bytes.  usage: python tools/mx_epi_check.py dump <out.npz> | cmp <a.npz> <b.npz>"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))

if sys.argv[1] == "cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    same = all(np.array_equal(a[k], b[k]) for k in ("c", "s"))
    print("identical" if same else "DIFFERENT", {k: int((a[k] != b[k]).sum()) for k in ("c", "s")})
    sys.exit(0 if same else 1)

import torch  # noqa: E402
from vcap import _native as N  # noqa: E402

dev = torch.device("cuda:0")
lib = N.lib()
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device=dev).manual_seed(5)
M, Nn, K = 25216 + 77, 3072, 768      # a partial last row tile too


def quant(x):
    rows, kk = x.shape
    q = torch.empty(rows, kk, dtype=torch.uint8, device=dev)
    sc = torch.empty(int(lib.vcap_mx_scale_bytes(rows, kk)), dtype=torch.uint8, device=dev)
    N.check(lib.vcap_mx_quantize(N.DT_F32, x.data_ptr(), kk, rows, kk, q.data_ptr(), sc.data_ptr(), s), "q")
    return q, sc


A = torch.randn(M, K, generator=g, device=dev)
W = torch.randn(Nn, K, generator=g, device=dev) * 0.05
bias = torch.randn(Nn, generator=g, device=dev) * 0.1
aq, asc = quant(A)
wq, wsc = quant(W)
C = torch.zeros(M, Nn, dtype=torch.uint8, device=dev)
cs = torch.zeros(int(lib.vcap_mx_scale_bytes(M, Nn)), dtype=torch.uint8, device=dev)
N.check(lib.vcap_gemm_mx(aq.data_ptr(), asc.data_ptr(), wq.data_ptr(), wsc.data_ptr(), N.DT_MXFP8, C.data_ptr(), Nn,
                         cs.data_ptr(), M, Nn, K, bias.data_ptr(), 1, None, s), "gemm_mx")
torch.cuda.synchronize()
np.savez(sys.argv[2], c=C.cpu().numpy(), s=cs.cpu().numpy())
print("dumped", sys.argv[2])
