"""The fused QKV projection + attention (vcap_vit_qkv_attention, csrc/vit_attention.hip) is bit-identical
to the unfused pair it replaces in the bf16 encoder - vcap_gemm (bias, bf16 out) into a qkv buffer, then
vcap_vit_attention (timm Attention.qkv + the attention core, src/models/video_encoder.py:112-121) - for
every token row and for the class-token-only form of the last block, over frame counts that do and do not
take the XCD-aware workgroup order (frames % 8), token counts across both supported ranges (ViT-B/16's
193-208 and ViT-L/14's 257-272: vcap_vit_qkv_attention_l_kernel) and head counts other than 12 / 16."""
import numpy as np
import pytest
import torch

from vcap import _native as N

pytestmark = pytest.mark.gpu


def _s():
    return torch.cuda.current_stream().cuda_stream


def _case(device, BT, NT, H, seed):
    D = H * 64
    g = torch.Generator(device=device).manual_seed(seed)
    xn = torch.randn(BT * NT, D, generator=g, device=device).to(torch.bfloat16)
    w = (0.05 * torch.randn(3 * D, D, generator=g, device=device)).to(torch.bfloat16)
    b = 0.05 * torch.randn(3 * D, generator=g, device=device)
    return xn, w, b


def _unfused(xn, w, b, BT, NT, H):
    D = H * 64
    qkv = torch.empty(BT * NT, 3 * D, device=xn.device, dtype=torch.bfloat16)
    out = torch.empty(BT * NT, D, device=xn.device, dtype=torch.bfloat16)
    lib = N.lib()
    N.check(lib.vcap_gemm(N.DT_BF16, N.DT_BF16, xn.data_ptr(), D, w.data_ptr(), D, qkv.data_ptr(), 3 * D, BT * NT,
                          3 * D, D, b.data_ptr(), 0, None, 0, 0, 0, 0, 0, 0, _s()), "qkv gemm")
    N.check(lib.vcap_vit_attention(N.DT_BF16, qkv.data_ptr(), out.data_ptr(), BT, NT, H, _s()), "attention")
    return out


def _fused(xn, w, b, BT, NT, H, cls_only):
    out = torch.full((BT * NT, H * 64), float("nan"), device=xn.device, dtype=torch.bfloat16)
    N.check(N.lib().vcap_vit_qkv_attention(xn.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr(), BT, NT, H,
                                           cls_only, _s()), "qkv_attention")
    return out


@pytest.mark.parametrize("BT,NT,H", [(16, 197, 12), (5, 197, 12), (8, 208, 12), (3, 193, 12), (8, 200, 4),
                                     (2, 197, 1), (8, 257, 16), (3, 257, 16), (4, 272, 16), (2, 260, 4),
                                     (16, 257, 16)])
def test_fused_bit_identical(device, BT, NT, H):
    xn, w, b = _case(device, BT, NT, H, BT * 1000 + NT + H)
    ref = _unfused(xn, w, b, BT, NT, H)
    out = _fused(xn, w, b, BT, NT, H, 0)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16)), float((out.float() - ref.float()).abs().max())
    cls = _fused(xn, w, b, BT, NT, H, 1)
    torch.cuda.synchronize()
    want = ref.view(BT, NT, H * 64)[:, 0].contiguous()
    assert torch.equal(cls[:BT].view(torch.int16), want.view(torch.int16))
    assert torch.isnan(cls[BT:].float()).all()   # nothing written past the compact class-token rows


def test_fused_vs_fp32_sdpa(device):
    """Against fp32 SDPA over the bf16-rounded q / k / v of an fp32 qkv Linear (timm's Attention on the
    bf16 operands): what is left is the attention's bf16 P, the tolerance class of tests/test_gpu_bf16.py."""
    BT, NT, H = 4, 197, 12
    xn, w, b = _case(device, BT, NT, H, 7)
    out = _fused(xn, w, b, BT, NT, H, 0).float()
    qkv = (xn.float() @ w.float().t() + b).to(torch.bfloat16).float()   # q / k / v are bf16 on chip too
    q, k, v = qkv.view(BT, NT, 3, H, 64).permute(2, 0, 3, 1, 4)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v).permute(0, 2, 1, 3).reshape(BT * NT, H * 64)
    err = (out - ref).abs().max().item()
    assert err < 1e-2, err
    assert np.isfinite(out.cpu().numpy()).all()


def test_fused_refuses_other_shapes(device):
    xn, w, b = _case(device, 2, 197, 12, 1)
    lib = N.lib()
    for nt in (192, 209, 256, 273):
        assert lib.vcap_vit_qkv_attention(xn.data_ptr(), w.data_ptr(), b.data_ptr(), xn.data_ptr(), 2, nt, 12, 0,
                                          _s()) == N.E_UNSUPPORTED
