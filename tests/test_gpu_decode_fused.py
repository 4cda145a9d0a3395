"""The fused c_attn + attention decode launch (csrc/decode.hip EPI_QKVA: the last workgroup to store a
head's q / k / v columns attends that head for every row; `sc1` hand-off, per-head arrival
counters) against the two-launch form (GenConfig.split_attention): token ids AND every step's raw
logits bit-identical, for the shapes the fusion covers (bf16, <= 16 rows, GPT-2 small / medium
widths, whole-chip and capped grids = 1 / 2 tiles per workgroup, greedy with processors, raw greedy,
a token prompt), across repeated graph replays (the counters are left zero by every launch) and
eagerly.  The two-launch form is itself the path the bf16 parity / fidelity tests pin to the
reference (tests/test_gpu_bf16.py, tests/test_gpu_fidelity.py)."""
import dataclasses

import numpy as np
import pytest
import torch

from helpers import case, state_dict
from vcap import configs, prng
from vcap.model import GenConfig, HipGPT2Decoder, HipPrefix, HipViTEncoder

pytestmark = pytest.mark.gpu
_CACHE = {}


def _prefix(device, name="b16_b8", B=None):
    meta, g, va, ga, sd, frames = case(name)
    key = ("pre", name)
    if key not in _CACHE:
        enc, pre = HipViTEncoder(sd, va, "bf16", device), HipPrefix(sd, ga.n_embd, device=device)
        _, prefix = enc.encode(torch.from_numpy(frames).to(device), pre)
        _CACHE[key] = (prefix, HipGPT2Decoder(sd, ga, "bf16", device), ga)
        del enc
    prefix, dec, ga = _CACHE[key]
    if B is not None:
        reps = -(-B // prefix.shape[0])
        prefix = prefix.repeat(reps, 1, 1)[:B].contiguous()
        # distinct rows: perturb the copies so each row decodes its own sequence
        prefix = prefix + 0.05 * torch.arange(B, device=device, dtype=prefix.dtype).view(B, 1, 1) / B
    return prefix, dec, ga


def _run(dec, ga, prefix, cfg, prompt=None):
    B, L = prefix.shape[0], cfg.max_new_tokens
    logits = torch.empty(L, B, ga.vocab, dtype=torch.float32, device=prefix.device)
    ids = dec.generate_ids(prefix, prompt or [ga.bos_token_id], cfg, logits_out=logits)
    torch.cuda.synchronize()
    return ids.cpu().numpy(), logits.cpu().numpy()


def _assert_same(dec, ga, prefix, cfg, prompt=None):
    ids0, lg0 = _run(dec, ga, prefix, dataclasses.replace(cfg, split_attention=True), prompt)
    ids1, lg1 = _run(dec, ga, prefix, dataclasses.replace(cfg, split_attention=False), prompt)
    assert np.array_equal(ids0, ids1)
    assert np.array_equal(lg0.view(np.int32), lg1.view(np.int32)), float(np.abs(lg0 - lg1).max())
    return ids1


@pytest.mark.parametrize("B", [1, 3, 8, 16])
@pytest.mark.parametrize("max_blocks", [0, 96])
def test_fused_equals_split_hf_greedy(device, B, max_blocks):
    prefix, dec, ga = _prefix(device, B=B)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    cfg.max_blocks = max_blocks
    _assert_same(dec, ga, prefix, cfg)


def test_fused_equals_split_raw_greedy_and_prompt(device):
    prefix, dec, ga = _prefix(device)
    _assert_same(dec, ga, prefix, GenConfig.raw_greedy(24, ga.eos_token_id, True))
    # a 7-token prompt: context 4 + 7 + 23 = 34 positions (three KV pages)
    _assert_same(dec, ga, prefix, GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True),
                 prompt=[464, 3797, 318, 257, 1310, 286, 50256])


def test_fused_eager_equals_graph(device):
    prefix, dec, ga = _prefix(device)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    ids_g, lg_g = _run(dec, ga, prefix, cfg)
    ids_e, lg_e = _run(dec, ga, prefix, dataclasses.replace(cfg, use_graph=False))
    assert np.array_equal(ids_g, ids_e) and np.array_equal(lg_g.view(np.int32), lg_e.view(np.int32))


def test_fused_repeated_replays_stay_identical(device):
    """50 replays of one captured fused decode: every replay's ids equal the first (a counter left
    non-zero by some launch would change which workgroup attends a head - or none would)."""
    prefix, dec, ga = _prefix(device)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    cfg.max_blocks = 96
    out = torch.empty(prefix.shape[0], 24, dtype=torch.int32, device=device)
    ref = dec.generate_ids(prefix, [ga.bos_token_id], cfg, out=out).cpu().numpy().copy()
    for _ in range(50):
        dec.generate_ids(prefix, [ga.bos_token_id], cfg, out=out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("B", [2, 8])
def test_fused_equals_split_gpt2_medium(device, B):
    """GPT-2-medium widths (E = 1024, 16 heads: the NSL = 8 instantiation)."""
    va, ga = configs.vit_arch("vit_large_patch14_224"), configs.gpt2_arch("gpt2-medium")
    sd = state_dict("vit_large_patch14_224", "gpt2-medium", 1)
    dec = HipGPT2Decoder(sd, ga, "bf16", device)
    g = torch.Generator().manual_seed(5)
    prefix = (0.5 * torch.randn(B, 4, ga.n_embd, generator=g)).to(device)
    _assert_same(dec, ga, prefix, GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True))
    del dec
    torch.cuda.empty_cache()
