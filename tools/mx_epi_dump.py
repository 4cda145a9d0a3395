"""Dump the fc1 MXFP8 epilogue output (e4m3 bytes + the scales of the valid rows) of whichever
library VCAP_LIB names, for a bit-exactness A/B of two builds:
  VCAP_LIB=a.so python tools/mx_epi_dump.py out_a.pt; VCAP_LIB=b.so python tools/mx_epi_dump.py out_b.pt
  python tools/mx_epi_dump.py --compare out_a.pt out_b.pt"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

if sys.argv[1] == "--compare":
    a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
    for k in a:
        same = torch.equal(a[k], b[k])
        print(f"{k}: {'identical' if same else 'DIFFERENT'} ({a[k].numel()} bytes)")
        assert same
    sys.exit(0)

from oracle import vcap_oracle as O  # noqa: E402  (test infrastructure: layout unpacking only)
from vcap import _native as N  # noqa: E402

dev = torch.device("cuda:0")
lib = N.lib()
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device=dev).manual_seed(0)
res = {}
for M in (600, 25216):
    Nn, K = 3072, 768
    A = torch.randn(M, K, generator=g, device=dev)
    W = torch.randn(Nn, K, generator=g, device=dev) * 0.05
    bias = torch.linspace(-0.5, 0.5, Nn, device=dev)
    qs = []
    for x in (A, W):
        q = torch.empty(x.shape, dtype=torch.uint8, device=dev)
        sc = torch.empty(int(lib.vcap_mx_scale_bytes(x.shape[0], K)), dtype=torch.uint8, device=dev)
        N.check(lib.vcap_mx_quantize(N.DT_F32, x.data_ptr(), K, x.shape[0], K, q.data_ptr(), sc.data_ptr(), s), "q")
        qs += [q, sc]
    c = torch.empty(M, Nn, dtype=torch.uint8, device=dev)
    csc = torch.zeros(int(lib.vcap_mx_scale_bytes(M, Nn)), dtype=torch.uint8, device=dev)
    N.check(lib.vcap_gemm_mx(qs[0].data_ptr(), qs[1].data_ptr(), qs[2].data_ptr(), qs[3].data_ptr(), N.DT_MXFP8,
                             c.data_ptr(), Nn, csc.data_ptr(), M, Nn, K, bias.data_ptr(), 1, None, s), "gemm_mx")
    torch.cuda.synchronize()
    res[f"c{M}"] = c.cpu()
    res[f"s{M}"] = torch.from_numpy(O.mx_unpack_scales(csc.cpu().numpy(), M, Nn).copy())
torch.save(res, sys.argv[1])
print("saved", sys.argv[1], N.library_path())
