"""MXFP8 path (BASELINE configs[4]: fp8 MFMA for the ViT GEMMs) through the C ABI.

Oracle: oracle/vcap_oracle.py mx_quantize / mx_dequantize (OCP MXFP8-E4M3 restatement).
  * quantisation (weights, LayerNorm outputs): e4m3 bytes and E8M0 scales bit-identical to the
    oracle (LayerNorm: >= 99.9 % identical - the f32 statistics can differ in the last ulp and
    move a value across an e4m3 rounding boundary - and all within one e4m3 step);
  * GEMM: the scaled MFMA against float64 dequant(A) . dequant(W)^T, within 2e-4 of sum |a.b|;
  * GELU -> MXFP8 epilogue: within one e4m3 step of the quantised exact result;
  * full ViT-B/16 encoder in fp8 vs the reference's fp32 output (tests/golden/b16_b8): tolerance
    stated in the test (e4m3 keeps 3 mantissa bits: ~3 % relative per operand)."""
import numpy as np
import pytest
import torch

from helpers import case
from oracle import vcap_oracle as O
from vcap import _native as N

pytestmark = pytest.mark.gpu


def _s():
    return torch.cuda.current_stream().cuda_stream


def _quant_gpu(x: torch.Tensor):
    rows, K = x.shape
    q = torch.empty(rows, K, dtype=torch.uint8, device=x.device)
    sc = torch.zeros(int(N.lib().vcap_mx_scale_bytes(rows, K)), dtype=torch.uint8, device=x.device)
    dt = N.DT_F32 if x.dtype == torch.float32 else N.DT_BF16
    N.check(N.lib().vcap_mx_quantize(dt, x.data_ptr(), K, rows, K, q.data_ptr(), sc.data_ptr(), _s()), "quantize")
    return q, sc


def _rand(rows, K, seed, spread=True):
    g = np.random.default_rng(seed)
    x = g.standard_normal((rows, K)).astype(np.float32)
    if spread:  # block magnitudes over many binades, one all-zero block, a few tiny values
        x *= np.exp2(g.integers(-12, 12, (rows, K // 32, 1))).repeat(32, -1).reshape(rows, K).astype(np.float32)
        x[0, :32] = 0
        x[-1, 5] = 1e-30
    return x


@pytest.mark.parametrize("rows,K", [(1, 256), (300, 512), (2304, 768)])
def test_mx_quantize_bit_exact(device, rows, K):
    x = _rand(rows, K, rows)
    q, sc = _quant_gpu(torch.from_numpy(x).to(device))
    torch.cuda.synchronize()
    qo, so = O.mx_quantize(x)
    assert np.array_equal(O.mx_unpack_scales(sc.cpu().numpy(), rows, K), so)
    assert np.array_equal(q.cpu().numpy(), qo)


@pytest.mark.parametrize("M,N_,K", [(256, 256, 256), (300, 384, 512), (1000, 2304, 768), (777, 768, 3072)])
@pytest.mark.parametrize("out", ["bf16", "f32"])
def test_gemm_mx_matches_dequantized_product(device, M, N_, K, out):
    a, w = _rand(M, K, 1), _rand(N_, K, 2)
    aq, asc = _quant_gpu(torch.from_numpy(a).to(device))
    wq, wsc = _quant_gpu(torch.from_numpy(w).to(device))
    bias = torch.from_numpy(np.random.default_rng(3).standard_normal(N_).astype(np.float32)).to(device)
    odt, tdt = (N.DT_BF16, torch.bfloat16) if out == "bf16" else (N.DT_F32, torch.float32)
    c = torch.empty(M, N_, dtype=tdt, device=device)
    N.check(N.lib().vcap_gemm_mx(aq.data_ptr(), asc.data_ptr(), wq.data_ptr(), wsc.data_ptr(), odt, c.data_ptr(), N_,
                                 None, M, N_, K, bias.data_ptr(), 0, None, _s()), "gemm_mx")
    torch.cuda.synchronize()
    ad = O.mx_dequantize(aq.cpu().numpy(), O.mx_unpack_scales(asc.cpu().numpy(), M, K)).astype(np.float64)
    wd = O.mx_dequantize(wq.cpu().numpy(), O.mx_unpack_scales(wsc.cpu().numpy(), N_, K)).astype(np.float64)
    ref = ad @ wd.T + bias.cpu().numpy()
    got = c.float().cpu().numpy()
    scale = np.abs(ad) @ np.abs(wd).T + 1e-30  # error scale of an f32 (or bf16-rounded) sum
    rel = np.abs(got - ref) / scale
    # f32 out: the scaled MFMA's internal sum of fp8 products is not an f32 fma chain; measured
    # <= 1e-4 of sum |a.b| (vs ~1e-7 for bf16 MFMA) - far below e4m3's own 2^-4 operand rounding
    tol = 2e-4 if out == "f32" else 2 ** -8
    bad = rel > tol
    if bad.any():
        ratio = np.median(got[bad] / np.where(ref[bad] == 0, 1, ref[bad]))
        pytest.fail(f"{bad.sum()} / {bad.size} outside {tol}: max rel {rel.max():.3g}, median got/ref {ratio:.4g}")


def test_gemm_mx_residual_in_place(device):
    M, N_, K = 520, 768, 3072
    a, w = _rand(M, K, 4, spread=False), _rand(N_, K, 5, spread=False)
    aq, asc = _quant_gpu(torch.from_numpy(a).to(device))
    wq, wsc = _quant_gpu(torch.from_numpy(w).to(device))
    bias = torch.linspace(-1, 1, N_, device=device)
    x0 = torch.randn(M, N_, device=device)
    x = x0.clone()
    N.check(N.lib().vcap_gemm_mx(aq.data_ptr(), asc.data_ptr(), wq.data_ptr(), wsc.data_ptr(), N.DT_F32, x.data_ptr(),
                                 N_, None, M, N_, K, bias.data_ptr(), 0, x.data_ptr(), _s()), "gemm_mx")
    torch.cuda.synchronize()
    ad = O.mx_dequantize(aq.cpu().numpy(), O.mx_unpack_scales(asc.cpu().numpy(), M, K)).astype(np.float64)
    wd = O.mx_dequantize(wq.cpu().numpy(), O.mx_unpack_scales(wsc.cpu().numpy(), N_, K)).astype(np.float64)
    ref = x0.cpu().numpy() + ad @ wd.T + bias.cpu().numpy()
    scale = np.abs(ad) @ np.abs(wd).T + np.abs(x0.cpu().numpy()) + 1e-30
    assert (np.abs(x.cpu().numpy() - ref) / scale).max() < 2e-4


def _e4m3_step(sbytes):
    """one e4m3 step at the top binade of a block: 2^(scale-127) * 16 (values in [128, 256))"""
    return np.exp2(sbytes.astype(np.float64) - 127.0) * 16.0


def test_gemm_mx_gelu_to_mxfp8(device):
    """fc1 epilogue: bias + GELU-tanh, re-quantised to MXFP8 for fc2."""
    M, N_, K = 600, 3072, 768
    a, w = _rand(M, K, 6, spread=False), _rand(N_, K, 7, spread=False) * 0.05
    aq, asc = _quant_gpu(torch.from_numpy(a).to(device))
    wq, wsc = _quant_gpu(torch.from_numpy(w).to(device))
    bias = torch.linspace(-0.5, 0.5, N_, device=device)
    c = torch.empty(M, N_, dtype=torch.uint8, device=device)
    csc = torch.zeros(int(N.lib().vcap_mx_scale_bytes(M, N_)), dtype=torch.uint8, device=device)
    N.check(N.lib().vcap_gemm_mx(aq.data_ptr(), asc.data_ptr(), wq.data_ptr(), wsc.data_ptr(), N.DT_MXFP8, c.data_ptr(),
                                 N_, csc.data_ptr(), M, N_, K, bias.data_ptr(), 1, None, _s()), "gemm_mx gelu")
    torch.cuda.synchronize()
    ad = O.mx_dequantize(aq.cpu().numpy(), O.mx_unpack_scales(asc.cpu().numpy(), M, K)).astype(np.float64)
    wd = O.mx_dequantize(wq.cpu().numpy(), O.mx_unpack_scales(wsc.cpu().numpy(), N_, K)).astype(np.float64)
    h = torch.from_numpy(ad @ wd.T + bias.cpu().numpy().astype(np.float64))
    ref = torch.nn.functional.gelu(h, approximate="tanh").float().numpy()
    qo, so = O.mx_quantize(ref)
    sg = O.mx_unpack_scales(csc.cpu().numpy(), M, N_)
    assert (sg == so).mean() > 0.999
    got = O.mx_dequantize(c.cpu().numpy(), sg)
    step = np.repeat(_e4m3_step(so), 32, axis=1)
    assert (np.abs(got - O.mx_dequantize(qo, so)) <= step + 1e-12).all()


def test_layernorm_mx(device):
    rows, D = 1000, 768
    x = torch.randn(rows, D, device=device) * 3 + 1
    g = torch.rand(D, device=device) + 0.5
    b = torch.randn(D, device=device) * 0.1
    q = torch.empty(rows, D, dtype=torch.uint8, device=device)
    sc = torch.zeros(int(N.lib().vcap_mx_scale_bytes(rows, D)), dtype=torch.uint8, device=device)
    N.check(N.lib().vcap_layernorm_mx(x.data_ptr(), D, q.data_ptr(), sc.data_ptr(), g.data_ptr(), b.data_ptr(), rows, D,
                                      1e-6, _s()), "layernorm_mx")
    torch.cuda.synchronize()
    ref = torch.nn.functional.layer_norm(x.cpu().double(), (D,), g.cpu().double(), b.cpu().double(), 1e-6).float().numpy()
    qo, so = O.mx_quantize(ref)
    sg = O.mx_unpack_scales(sc.cpu().numpy(), rows, D)
    assert (sg == so).mean() > 0.999
    assert (q.cpu().numpy() == qo).mean() > 0.999
    got = O.mx_dequantize(q.cpu().numpy(), sg)
    assert (np.abs(got - O.mx_dequantize(qo, so)) <= np.repeat(_e4m3_step(so), 32, axis=1) + 1e-12).all()


@pytest.mark.parametrize("name,tol", [("b16_b8", 0.25), ("l14_medium", 0.35)])
def test_encoder_fp8_close_to_reference(device, name, tol):
    """fp8 (MXFP8 QKV / fc1 / fc2) ViT encoder vs the reference's fp32 encoder output.  Stated
    tolerance: max |err| < tol on outputs of O(1) magnitude and cosine similarity > 0.995 per
    video (e4m3 rounding of three GEMM operands per block; bf16 mode is within 3e-2)."""
    from vcap.model import HipPrefix, HipViTEncoder
    meta, g, va, ga, sd, frames = case(name)
    enc = HipViTEncoder(sd, va, "fp8", device)
    out, _ = enc.encode(torch.from_numpy(frames).to(device), HipPrefix(sd, ga.n_embd, device=device))
    got, ref = out.cpu().numpy().astype(np.float64), g["encoder_out"].astype(np.float64)
    err = np.abs(got - ref).max()
    cos = (got * ref).sum(1) / np.linalg.norm(got, axis=1) / np.linalg.norm(ref, axis=1)
    print(f"{name}: fp8 encoder max|err| {err:.4f} (ref max {np.abs(ref).max():.3f}), min cos {cos.min():.6f}")
    assert err < tol and cos.min() > 0.995, (err, cos.min())


@pytest.mark.parametrize("tokens,heads", [(197, 12), (257, 16)])
def test_attention_mx_output(device, tokens, heads):
    """MXFP8 attention output vs the bf16 attention output of the same kernel arithmetic: every
    element within half an e4m3 step of the bf16 value (+ the bf16 rounding), scales equal except
    where the bf16 rounding lifts a block max across a power of two."""
    frames, D = 6, heads * 64
    g = torch.Generator(device=device).manual_seed(0)
    qkv = (torch.randn(frames * tokens, 3 * D, generator=g, device=device) * 1.5).bfloat16()
    ref = torch.empty(frames * tokens, D, dtype=torch.bfloat16, device=device)
    N.check(N.lib().vcap_vit_attention(N.DT_BF16, qkv.data_ptr(), ref.data_ptr(), frames, tokens, heads, _s()), "attn")
    M = frames * tokens
    q = torch.empty(M, D, dtype=torch.uint8, device=device)
    sc = torch.zeros(int(N.lib().vcap_mx_scale_bytes(M, D)), dtype=torch.uint8, device=device)
    N.check(N.lib().vcap_vit_attention_mx(qkv.data_ptr(), q.data_ptr(), sc.data_ptr(), frames, tokens, heads, _s()),
            "attn mx")
    torch.cuda.synchronize()
    r = ref.float().cpu().numpy().astype(np.float64)
    qo, so = O.mx_quantize(ref.float().cpu().numpy())
    sg = O.mx_unpack_scales(sc.cpu().numpy(), M, D)
    # a block max just below a power of two can round up to it in bf16: the scale then differs by 1
    assert (sg == so).mean() > 0.99 and (np.abs(sg.astype(int) - so.astype(int)) <= 1).all()
    got = O.mx_dequantize(q.cpu().numpy(), sg)
    half_step = np.repeat(_e4m3_step(sg) / 2, 32, axis=1)
    assert (np.abs(got - r) <= half_step + np.abs(r) * 2.0 ** -8 + 1e-12).all()


# Caption-level fidelity of the MXFP8 encoder (configs[4]): tests/test_gpu_fidelity.py
# (test_fp8_divergences_are_near_ties: every divergence explained by an fp32 near-tie, leading-token
# agreement at least the floor the margins guarantee; the r02 measured floor is retired).
