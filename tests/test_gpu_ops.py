"""Per-kernel parity: each HIP entry point of include/vcap.h against a plain PyTorch fp32
reference of the same op, on seeded inputs (edge shapes: rows not a multiple of the tile,
197/257 tokens, B=1).  Tolerances: fp32 mode 1e-4 relative-ish (MFMA f32 FMA chains in a
different order than rocBLAS/CPU), bf16 mode compares against an fp32 reference fed the
same bf16-rounded operands."""
import ctypes as C

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from vcap import _native as N

pytestmark = pytest.mark.gpu


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _rand(shape, seed, scale=1.0, device="cuda"):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(device)


@pytest.fixture(params=[1, 2], ids=["tile128", "tile256"])
def gemm_policy(request):
    """Run a GEMM test with the 128x128 kernel and again with the 256x256 8-phase kernel forced
    wherever its shape constraints hold (vcap_set_gemm_policy)."""
    N.check(N.lib().vcap_set_gemm_policy(request.param), "policy")
    yield request.param
    N.check(N.lib().vcap_set_gemm_policy(0), "policy")


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("M,N_,K", [(300, 384, 256), (128, 128, 64), (1, 2304, 768), (197, 200, 192),
                                    (3152, 2304, 768), (1000, 768, 3072), (257, 272, 128)])
def test_gemm_plain_bias(device, gemm_policy, prec, M, N_, K):
    dt, tdt = (N.DT_F32, torch.float32) if prec == "fp32" else (N.DT_BF16, torch.bfloat16)
    if prec == "bf16" and K % 64:
        pytest.skip("bf16 K step is 64")
    A = _rand((M, K), 1).to(tdt)
    W = _rand((N_, K), 2, 0.05).to(tdt)
    b = _rand((N_,), 3, 0.1)
    out = torch.empty(M, N_, dtype=tdt, device=device)
    N.check(N.lib().vcap_gemm(dt, dt, A.data_ptr(), K, W.data_ptr(), K, out.data_ptr(), N_, M, N_, K, b.data_ptr(),
                              0, None, 0, 0, 0, 0, 0, 0, _stream()), "gemm")
    ref = A.float() @ W.float().t() + b
    tol = 2e-4 if prec == "fp32" else 2e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_gemm_gelu_and_residual(device, gemm_policy, prec):
    dt, tdt = (N.DT_F32, torch.float32) if prec == "fp32" else (N.DT_BF16, torch.bfloat16)
    M, N_, K = 333, 256, 128
    A = _rand((M, K), 4).to(tdt)
    W = _rand((N_, K), 5, 0.1).to(tdt)
    b = _rand((N_,), 6, 0.1)
    g = torch.empty(M, N_, dtype=tdt, device=device)
    N.check(N.lib().vcap_gemm(dt, dt, A.data_ptr(), K, W.data_ptr(), K, g.data_ptr(), N_, M, N_, K, b.data_ptr(), 1,
                              None, 0, 0, 0, 0, 0, 0, _stream()), "gemm gelu")
    ref = F.gelu(A.float() @ W.float().t() + b, approximate="tanh")
    tol = 2e-4 if prec == "fp32" else 2e-2
    torch.testing.assert_close(g.float(), ref, rtol=tol, atol=tol)
    # in-place residual into an f32 stream
    x = _rand((M, N_), 7)
    x0 = x.clone()
    N.check(N.lib().vcap_gemm(dt, N.DT_F32, A.data_ptr(), K, W.data_ptr(), K, x.data_ptr(), N_, M, N_, K,
                              b.data_ptr(), 0, x.data_ptr(), N_, 1, 0, 0, 0, 0, _stream()), "gemm resid")
    torch.testing.assert_close(x, x0 + A.float() @ W.float().t() + b, rtol=tol, atol=tol)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_gemm_patch_remap_pos(device, gemm_policy, prec):
    """Patch-embed epilogue: out row (m/P)*(P+1)+1+m%P, + bias + pos[1 + m%P]."""
    dt, tdt = (N.DT_F32, torch.float32) if prec == "fp32" else (N.DT_BF16, torch.bfloat16)
    BT, P, D, K = 3, 196, 128, 768
    A = _rand((BT * P, K), 8).to(tdt)
    W = _rand((D, K), 9, 0.02).to(tdt)
    b = _rand((D,), 10, 0.1)
    pos = _rand((P + 1, D), 11, 0.1)
    x = torch.zeros(BT * (P + 1), D, device=device)
    N.check(N.lib().vcap_gemm(dt, N.DT_F32, A.data_ptr(), K, W.data_ptr(), K, x.data_ptr(), D, BT * P, D, K,
                              b.data_ptr(), 0, pos.data_ptr(), D, 2, P, P + 1, 1, 1, _stream()), "gemm patch")
    ref = (A.float() @ W.float().t() + b).reshape(BT, P, D) + pos[1:]
    got = x.reshape(BT, P + 1, D)
    tol = 2e-4 if prec == "fp32" else 2e-2
    torch.testing.assert_close(got[:, 1:], ref, rtol=tol, atol=tol)
    assert float(got[:, 0].abs().max()) == 0.0


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("rows,D,eps,affine", [(197, 768, 1e-6, True), (5, 1024, 1e-5, True), (3, 256, 1e-5, False),
                                               (7, 128, 1e-6, True)])
def test_layernorm(device, prec, rows, D, eps, affine):
    dt, tdt = (N.DT_F32, torch.float32) if prec == "fp32" else (N.DT_BF16, torch.bfloat16)
    x = _rand((rows, D), 12, 2.0) + 0.5
    g = _rand((D,), 13, 0.1) + 1 if affine else None
    b = _rand((D,), 14, 0.1) if affine else None
    y = torch.empty(rows, D, dtype=tdt, device=device)
    N.check(N.lib().vcap_layernorm(dt, x.data_ptr(), D, y.data_ptr(), D, N.ptr(g), N.ptr(b), rows, D, eps,
                                   _stream()), "layernorm")
    ref = F.layer_norm(x, (D,), g, b, eps)
    tol = 1e-5 if prec == "fp32" else 1e-2
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("BT,Ntok,H", [(3, 197, 2), (1, 257, 16), (2, 197, 12)])
def test_vit_attention(device, prec, BT, Ntok, H):
    dt, tdt = (N.DT_F32, torch.float32) if prec == "fp32" else (N.DT_BF16, torch.bfloat16)
    D = H * 64
    qkv = _rand((BT * Ntok, 3 * D), 15, 1.5).to(tdt)
    out = torch.empty(BT * Ntok, D, dtype=tdt, device=device)
    N.check(N.lib().vcap_vit_attention(dt, qkv.data_ptr(), out.data_ptr(), BT, Ntok, H, _stream()), "attention")
    q, k, v = qkv.float().reshape(BT, Ntok, 3, H, 64).permute(2, 0, 3, 1, 4).unbind(0)
    ref = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(BT * Ntok, D)
    tol = 1e-4 if prec == "fp32" else 3e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("gap", [0, 1])
def test_vit_pool_temporal(device, prec, gap):
    """core/operators/cupy_vit_pool.py:23-104 semantics."""
    dt, tdt = (N.DT_F32, torch.float32) if prec == "fp32" else (N.DT_BF16, torch.bfloat16)
    B, T, tok, Cc = 2, 3, 197, 768
    x = _rand((B * T, tok, Cc), 16).to(tdt)
    y = torch.empty(B, Cc, dtype=tdt, device=device)
    N.check(N.lib().vcap_vit_pool_temporal(dt, x.data_ptr(), y.data_ptr(), B, T, tok, Cc, gap, _stream()), "pool")
    xb = x.float().reshape(B, T, tok, Cc)
    ref = xb[:, :, 0].mean(1) if not gap else xb[:, :, 1:].mean(dim=(1, 2))
    tol = 1e-5 if prec == "fp32" else 1e-2
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("ln_scale,in_weight", [(0.6, 0.4), (0.0, 0.0), (0.6, 0.0)])
def test_prefix_project(device, ln_scale, in_weight):
    """core/engine.py:44-50 + mapper Linear(256 -> 4*768)."""
    B = 3
    emb = _rand((B, 256), 17)
    w = _rand((3072, 256), 18, 0.06)
    b = _rand((3072,), 19, 0.06)
    pd = N.PrefixDesc(ln_scale=ln_scale, in_weight=in_weight, prefix_len=4, n_embd=768, mapper_w=w.data_ptr(),
                      mapper_b=b.data_ptr())
    out = torch.empty(B, 4, 768, device=device)
    N.check(N.lib().vcap_prefix_project(emb.data_ptr(), B, 256, C.byref(pd), out.data_ptr(), _stream()), "prefix")
    e = emb
    if ln_scale > 0:
        e = F.layer_norm(e, (256,)) * ln_scale
    if in_weight > 0:
        e = e * in_weight
    ref = (e @ w.t() + b).reshape(B, 4, 768)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_linear_bias_matches_cupy_semantics(device, prec):
    """vcap_linear_bias: y[r,c] = b[c] + sum_k x[r,k] W[c,k] (cupy_linear_mapper.py:14-40)."""
    dt, tdt = (N.DT_F32, torch.float32) if prec == "fp32" else (N.DT_BF16, torch.bfloat16)
    x = _rand((5, 256), 20).to(tdt)
    w = _rand((3072, 256), 21, 0.05).to(tdt)
    b = _rand((3072,), 22, 0.05)
    y = torch.empty(5, 3072, dtype=tdt, device=device)
    N.check(N.lib().vcap_linear_bias(dt, x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), 5, 256, 3072,
                                     _stream()), "linear_bias")
    tol = 2e-4 if prec == "fp32" else 2e-2
    torch.testing.assert_close(y.float(), x.float() @ w.float().t() + b, rtol=tol, atol=tol)


def test_abi_errors_are_reported(device):
    lib = N.lib()
    rc = lib.vcap_gemm(N.DT_BF16, N.DT_BF16, 1, 100, 1, 100, 1, 100, 4, 4, 100, None, 0, None, 0, 0, 0, 0, 0, 0,
                       _stream())
    assert rc != 0 and b"K" in lib.vcap_last_error()
    assert lib.vcap_vit_attention(N.DT_F32, 1, 1, 1, 300, 1, _stream()) != 0


@pytest.mark.parametrize("M,K", [(25216, 768), (25216, 3072), (20000, 3072)])
def test_gemm_inplace_residual_auto_policy(device, M, K):
    """attn-proj / fc2 shapes under the auto policy: whole 256x256 rounds plus the split-K
    remainder (partials + reduce) - bf16 operands, f32 residual stream updated in place."""
    N_ = 768
    N.check(N.lib().vcap_set_gemm_policy(0), "policy")
    A = _rand((M, K), 21).to(torch.bfloat16)
    W = _rand((N_, K), 22, 0.03).to(torch.bfloat16)
    b = _rand((N_,), 23, 0.1)
    x = _rand((M, N_), 24)
    ref = x + A.float() @ W.float().t() + b
    N.check(N.lib().vcap_gemm(N.DT_BF16, N.DT_F32, A.data_ptr(), K, W.data_ptr(), K, x.data_ptr(), N_, M, N_, K,
                              b.data_ptr(), 0, x.data_ptr(), N_, 1, 0, 0, 0, 0, _stream()), "gemm resid")
    torch.testing.assert_close(x, ref, rtol=1e-4, atol=2e-4)   # f32 accumulation of bf16 products
