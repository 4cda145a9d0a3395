"""Dump the outputs of the 256x256 GEMM (policy 2) at the ViT shapes - bf16 QKV / fc1 + GELU, f32
fc2 + in-place residual, odd M and N - and of the MXFP8 fc1 epilogue, for a bit-exactness A/B of
two builds (the K accumulation order is part of the contract of a schedule change):
  VCAP_LIB=a.so python tools/gemm_dump.py a.pt; python tools/gemm_dump.py b.pt
  python tools/gemm_dump.py --compare a.pt b.pt"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import torch  # noqa: E402

if sys.argv[1] == "--compare":
    a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    for k in a:
        d = ""
        if k in bad:
            x, y = a[k].float(), b[k].float()
            d = f" max |diff| {(x - y).abs().max().item():.3g}, {(x != y).sum().item()} elements differ"
        print(f"{k}: {'DIFFERENT' if k in bad else 'identical'} ({a[k].numel()} elements){d}")
    sys.exit(1 if bad else 0)

from vcap import _native as N  # noqa: E402

dev = torch.device("cuda:0")
lib = N.lib()
N.check(lib.vcap_set_gemm_policy(2), "policy")
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device=dev).manual_seed(0)
res = {}
for name, M, n, k, f32, act in (("qkv", 25216, 2304, 768, False, 0), ("fc1", 25216, 3072, 768, False, 1),
                                ("fc2", 25216, 768, 3072, True, 0), ("odd", 1000, 272, 256, True, 0),
                                ("fc1_512", 600, 3072, 512, False, 1)):
    A = (torch.randn(M, k, generator=g, device=dev)).bfloat16()
    W = (torch.randn(n, k, generator=g, device=dev) * 0.05).bfloat16()
    b = torch.randn(n, generator=g, device=dev) * 0.1
    C = torch.randn(M, n, generator=g, device=dev) if f32 else torch.empty(M, n, device=dev, dtype=torch.bfloat16)
    N.check(lib.vcap_gemm(N.DT_BF16, N.DT_F32 if f32 else N.DT_BF16, A.data_ptr(), k, W.data_ptr(), k, C.data_ptr(),
                          n, M, n, k, b.data_ptr(), act, C.data_ptr() if f32 else None, n if f32 else 0,
                          1 if f32 else 0, 0, 0, 0, 0, s), name)
    torch.cuda.synchronize()
    res[name] = C.cpu()
A = torch.randn(3000, 768, generator=g, device=dev)
W = torch.randn(2304, 768, generator=g, device=dev) * 0.05
C = torch.empty(3000, 2304, device=dev)
N.check(lib.vcap_gemm(N.DT_F32, N.DT_F32, A.data_ptr(), 768, W.data_ptr(), 768, C.data_ptr(), 2304, 3000, 2304, 768,
                      None, 1, None, 0, 0, 0, 0, 0, 0, s), "f32")
torch.cuda.synchronize()
res["f32"] = C.cpu()
for M in (600, 25216):
    Nn, K = 3072, 768
    qs = []
    for x in (torch.randn(M, K, generator=g, device=dev), torch.randn(Nn, K, generator=g, device=dev) * 0.05):
        q = torch.empty(x.shape, dtype=torch.uint8, device=dev)
        sc = torch.empty(int(lib.vcap_mx_scale_bytes(x.shape[0], K)), dtype=torch.uint8, device=dev)
        N.check(lib.vcap_mx_quantize(N.DT_F32, x.data_ptr(), K, x.shape[0], K, q.data_ptr(), sc.data_ptr(), s), "q")
        qs += [q, sc]
    bias = torch.linspace(-0.5, 0.5, Nn, device=dev)
    c = torch.empty(M, Nn, dtype=torch.uint8, device=dev)
    csc = torch.zeros(int(lib.vcap_mx_scale_bytes(M, Nn)), dtype=torch.uint8, device=dev)
    N.check(lib.vcap_gemm_mx(qs[0].data_ptr(), qs[1].data_ptr(), qs[2].data_ptr(), qs[3].data_ptr(), N.DT_MXFP8,
                             c.data_ptr(), Nn, csc.data_ptr(), M, Nn, K, bias.data_ptr(), 1, None, s), "gemm_mx")
    c2 = torch.empty(M, Nn, dtype=torch.bfloat16, device=dev)
    N.check(lib.vcap_gemm_mx(qs[0].data_ptr(), qs[1].data_ptr(), qs[2].data_ptr(), qs[3].data_ptr(), N.DT_BF16,
                             c2.data_ptr(), Nn, None, M, Nn, K, bias.data_ptr(), 0, None, s), "gemm_mx bf16")
    torch.cuda.synchronize()
    res[f"mx{M}"] = c.cpu()
    res[f"mxs{M}"] = csc.cpu()
    res[f"mxbf{M}"] = c2.cpu()
torch.save(res, sys.argv[1])
print("saved", sys.argv[1], N.library_path())
