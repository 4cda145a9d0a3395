"""The f32 decoder's greedy steps take their token from a bf16 lm_head screen plus an f32 rescoring of
every token the screen's error bound cannot rule out (csrc/decode.hip vcap_decode_finalize_kernel<float,
true>, include/vcap.h vcap_gpt2_desc.lm_head_screen): the ids equal those of the full f32 lm_head
(the same decoder asked for raw logits, which runs the f32 lm_head, and a decoder built without the
screen) for HF-greedy and raw-greedy configurations, 1 / 8 / 16 rows and grid caps, and when many
tokens tie at the maximum (copies of the winning wte row: the lowest id must win, as in the f32 argmax)."""
import numpy as np
import pytest
import torch

from vcap import configs, weights
from vcap.model import GenConfig, HipGPT2Decoder

pytestmark = pytest.mark.gpu
WTE = "decoder.model.transformer.wte.weight"


@pytest.fixture(scope="module")
def ga():
    return configs.gpt2_arch("gpt2")


@pytest.fixture(scope="module")
def sd(ga):
    return weights.synthetic_gpt2(3, ga)


def _prefix(device, B, ga, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    return torch.randn(B, 4, ga.n_embd, generator=g, device=device) * 0.1


def _ids(dec, pre, ga, cfg, logits=False):
    out = None
    if logits:
        out = torch.empty(cfg.max_new_tokens, pre.shape[0], ga.vocab, dtype=torch.float32, device=pre.device)
    ids = dec.generate_ids(pre, [ga.bos_token_id], cfg, logits_out=out)
    torch.cuda.synchronize()
    return ids.cpu().numpy()


def _cfgs(ga, cap):
    hf = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    hf.max_blocks = cap
    raw = GenConfig.raw_greedy(24, ga.eos_token_id, True)
    raw.max_blocks = cap
    return {"hf": hf, "raw": raw}


@pytest.mark.parametrize("B,cap", [(1, 0), (8, 0), (16, 96)])
def test_screen_ids_equal_full_f32(device, sd, ga, B, cap):
    scr = HipGPT2Decoder(sd, ga, "fp32", device)
    full = HipGPT2Decoder(sd, ga, "fp32", device, screen=False)
    assert scr.screen and not full.screen
    pre = _prefix(device, B, ga, 100 + B)
    for name, cfg in _cfgs(ga, cap).items():
        a = _ids(scr, pre, ga, cfg)
        b = _ids(full, pre, ga, cfg)
        c = _ids(scr, pre, ga, cfg, logits=True)   # raw logits requested: the f32 lm_head runs
        assert np.array_equal(a, b), (name, a, b)
        assert np.array_equal(a, c), name


def test_screen_ties_take_the_lowest_id(device, sd, ga):
    """41 copies of the step-0 winner's wte row (ids lo .. lo+40) tie exactly in every f32 score:
    the f32 argmax keeps the lowest id, and so must the screen's rescoring of 41 candidates."""
    full0 = HipGPT2Decoder(sd, ga, "fp32", device, screen=False)
    pre = _prefix(device, 4, ga, 7)
    cfg = _cfgs(ga, 0)["hf"]
    t0 = int(_ids(full0, pre, ga, cfg)[0, 0])
    lo = t0 if t0 + 41 <= ga.vocab else t0 - 40
    sd2 = dict(sd)
    wte = np.array(sd[WTE], dtype=np.float32, copy=True)
    wte[lo: lo + 41] = wte[t0]
    sd2[WTE] = wte
    scr = HipGPT2Decoder(sd2, ga, "fp32", device)
    full = HipGPT2Decoder(sd2, ga, "fp32", device, screen=False)
    a, b = _ids(scr, pre, ga, cfg), _ids(full, pre, ga, cfg)
    assert np.array_equal(a, b), (a, b)
    assert a[0, 0] == lo   # the tie went to the lowest id
