"""Decode GEMV work splits are arithmetic-neutral: the residual projections' half-tile workgroups
(8 columns each, vcap_rows_gemm_dispatch `half`, used where the grid may double) and the wider tiles
a grid cap asks for give the same ids and bit-identical raw logits at every step as whole 16-column
tiles (grid cap 48: no half tiles; 4-tile workgroups for c_attn / c_fc).  The tiles only change
which workgroup computes a column; every column keeps its MFMA order and its split-K sum."""
import numpy as np
import pytest
import torch

from helpers import case
from vcap.model import GenConfig, HipGPT2Decoder, HipPrefix, HipViTEncoder

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def models(device):
    meta, g, va, ga, sd, frames = case("b16_b8")
    enc, pre = HipViTEncoder(sd, va, "bf16", device), HipPrefix(sd, ga.n_embd, device=device)
    _, prefix = enc.encode(torch.from_numpy(frames).to(device), pre)
    dec = {p: HipGPT2Decoder(sd, ga, p, device) for p in ("bf16", "fp32")}
    return ga, prefix, dec


def _run(dec, ga, prefix, cap):
    B = prefix.shape[0]
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    cfg.max_blocks = cap
    logits = torch.empty(24, B, ga.vocab, dtype=torch.float32, device=prefix.device)
    ids = dec.generate_ids(prefix, [ga.bos_token_id], cfg, logits_out=logits)
    torch.cuda.synchronize()
    return ids.cpu().numpy(), logits.cpu().numpy()


@pytest.mark.parametrize("prec", ["bf16", "fp32"])
@pytest.mark.parametrize("rows", [8, 16, 32])
def test_half_tiles_bit_identical(models, prec, rows):
    ga, prefix, dec = models
    pre = prefix.repeat(rows // prefix.shape[0], 1, 1).contiguous()
    pre = pre + 0.01 * torch.arange(rows, device=pre.device, dtype=pre.dtype).view(rows, 1, 1) / rows
    ref_ids, ref_lg = _run(dec[prec], ga, pre, 48)       # whole tiles everywhere
    for cap in (0, 96):                                   # half tiles for the residual projections
        ids, lg = _run(dec[prec], ga, pre, cap)
        assert np.array_equal(ids, ref_ids), cap
        assert np.array_equal(lg.view(np.int32), ref_lg.view(np.int32)), (cap, float(np.abs(lg - ref_lg).max()))
