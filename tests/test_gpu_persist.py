"""Persistent greedy decode (csrc/decode_persist.hip: token steps 1.. as ONE launch of G resident
workgroups with grid barriers between phases; opt-in, measured slower than the launch chain - DESIGN
§4) against the launch chain (decode.hip, one launch per kernel): ids AND every step's raw logits
bit-identical, at the bench shapes (B = 8 and 16 rows of GPT-2 small), raw greedy, GPT-2-medium and
the tiny config, for several grid sizes.  The launch chain itself is pinned to the reference
(test_gpu_bf16.py teacher-forced bf16, test_gpu_parity.py fp32 token-exact).  (Bit equality holds
because every decode kernel computes its LayerNorm through the same explicit-fma helpers,
vcap_common.h sumsq4 / ln_affine4: left to the compiler's FMA contraction, single rows differed by up
to 1.3e-2 from some step on - profiles/r04_persistent_decode.txt.)"""
import dataclasses

import numpy as np
import pytest
import torch

from helpers import case
from vcap import _native as N
from vcap import configs, prng, weights

pytestmark = pytest.mark.gpu
_DEC = {}


def _decoder(gpt2, seed, device):
    from vcap.model import HipGPT2Decoder
    key = (gpt2, seed)
    if key not in _DEC:
        _DEC.clear()
        ga = configs.gpt2_arch(gpt2)
        sd = weights.synthetic_state_dict(seed, configs.vit_arch("vit_tiny_test"), ga)
        _DEC[key] = (HipGPT2Decoder(sd, ga, "bf16", device), ga)
    return _DEC[key]


def _prefix(B, E, seed, device):
    g = np.random.default_rng(seed)
    return torch.from_numpy((g.standard_normal((B, 4, E)) * 0.5).astype(np.float32)).to(device)


def _run(dec, ga, prefix, cfg, prompt=None):
    L, B = cfg.max_new_tokens, prefix.shape[0]
    logits = torch.full((L, B, ga.vocab), float("nan"), device=prefix.device)
    ids = dec.generate_ids(prefix, prompt or [ga.bos_token_id], cfg, logits_out=logits)
    torch.cuda.synchronize()
    return ids.cpu().numpy(), logits


def _check(dec, ga, prefix, cfg, G, prompt=None):
    faults0 = N.lib().vcap_decode_faults()
    ids0, lg0 = _run(dec, ga, prefix, dataclasses.replace(cfg, persistent=0), prompt)
    ids1, lg1 = _run(dec, ga, prefix, dataclasses.replace(cfg, persistent=G), prompt)
    assert N.lib().vcap_decode_faults() == faults0, "a persistent-decode barrier timed out"
    assert np.array_equal(ids0, ids1)
    d = float((lg0 - lg1).abs().max())
    print(f"max |logit d| = {d:.3e}")
    assert torch.equal(lg0, lg1), d


@pytest.mark.parametrize("B", [8, 16])
@pytest.mark.parametrize("G", [96, 128, 256])
def test_persistent_equals_launch_chain_gpt2(device, B, G):
    from vcap.model import GenConfig
    dec, ga = _decoder("gpt2", 1, device)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    _check(dec, ga, _prefix(B, ga.n_embd, B + G, device), cfg, G)


def test_persistent_equals_launch_chain_golden_prefix(device):
    """The reference's own b16_b8 prefixes (tests/golden, make_goldens.py): the bf16 decode both ways."""
    from vcap.model import GenConfig, HipGPT2Decoder
    meta, g, va, ga, sd, frames = case("b16_b8")
    dec = HipGPT2Decoder(sd, ga, "bf16", device)
    prefix = torch.from_numpy(g["inputs_embeds"][:, :4].copy()).to(device)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    _check(dec, ga, prefix, cfg, 128)


def test_persistent_raw_greedy_and_prompt(device):
    """Raw greedy (processors off, benchmark_baseline.py:160-240) and a 7-token id prompt (S0 = 11)."""
    from vcap.model import GenConfig
    dec, ga = _decoder("gpt2", 1, device)
    _check(dec, ga, _prefix(8, ga.n_embd, 3, device), GenConfig.raw_greedy(24, ga.eos_token_id), 128)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    _check(dec, ga, _prefix(5, ga.n_embd, 4, device), cfg, 128, prompt=[16594, 257, 1790, 11, 3288, 8305, 25])


def test_persistent_eager_equals_graph(device):
    """Without hipGraph capture (use_graph False) the persistent launch runs eagerly: same ids."""
    from vcap.model import GenConfig
    dec, ga = _decoder("gpt2", 1, device)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, False)
    _check(dec, ga, _prefix(8, ga.n_embd, 9, device), cfg, 128)


@pytest.mark.parametrize("gpt2,B", [("gpt2-medium", 8), ("gpt2_tiny_test", 16)])
def test_persistent_other_widths(device, gpt2, B):
    """GPT-2-medium (E = 1024, 24 layers, 40 steps as the `detailed` preset's length) and the tiny
    test config (E = 128, vocab 1024)."""
    from vcap.model import GenConfig
    dec, ga = _decoder(gpt2, 2, device)
    L = 40 if gpt2 == "gpt2-medium" else 24
    cfg = GenConfig(L, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    _check(dec, ga, _prefix(B, ga.n_embd, 11, device), cfg, 128)


def test_persistent_repeated_replays_stay_identical(device):
    """50 replays of one persistent graph (barrier counters re-zeroed by the graph's memset node
    every replay): ids identical every time, no barrier timeout."""
    from vcap.model import GenConfig
    dec, ga = _decoder("gpt2", 1, device)
    prefix = _prefix(16, ga.n_embd, 21, device)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True, persistent=128)
    faults0 = N.lib().vcap_decode_faults()
    out = torch.empty(16, 24, dtype=torch.int32, device=device)
    first = dec.generate_ids(prefix, [ga.bos_token_id], cfg, out=out).cpu().clone()
    for _ in range(50):
        dec.generate_ids(prefix, [ga.bos_token_id], cfg, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), first)
    assert N.lib().vcap_decode_faults() == faults0
