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


def _bf16(x):
    """Round-to-nearest-even to bf16 (what torch's .to(bfloat16) and v_cvt_pk_bf16_f32 do)."""
    b = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    b = (b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000
    return b.astype(np.uint32).view(np.float32)


def _adversarial_screen_sd(sd, ga, a_id=4000, b_id=9000, delta=0.002):
    """ln_f weight 0 and bias beta make every ln_f row EXACTLY beta, so the screen's bf16 operand
    h~ = bf16(beta) is chosen here; wte rows a and b sit on disjoint halves of the dims, with beta
    and the rows rounding DOWN in magnitude on a's half and UP on b's, so the screen over-rates a and
    under-rates b by ~2u * |h||w| each (u = 2^-8), the largest error the bound admits for rows on
    half the dims.  Every score is negative (the repetition penalty multiplies them by 1.1), b beats
    a by `delta` in exact arithmetic, and every other row scores far below both.
    Returns (state dict, numpy check values)."""
    E = ga.n_embd
    assert E == 768
    w0 = 2.0 ** -5
    dn, up = 1 + 0.49 * 2.0 ** -7, 1 + 0.51 * 2.0 ** -7      # round down / up to the bf16 grid
    Sa, Sb, j0 = np.arange(0, 384), np.arange(384, 767), 767
    beta = np.ones(E, np.float32)
    beta[Sa], beta[Sb] = dn, up
    wa = np.zeros(E, np.float32)
    wb = np.zeros(E, np.float32)
    wa[Sa] = -w0 * dn
    wb[Sb] = -w0 * up
    s_a = float(np.dot(beta.astype(np.float64), wa.astype(np.float64)))
    s_b0 = float(np.dot(beta.astype(np.float64), wb.astype(np.float64)))
    wb[j0] = _bf16(np.float32(s_a + delta - s_b0))       # bf16-exact tuning entry (beta[j0] = 1 exactly)
    kappa = np.float32(14.5 / beta.astype(np.float64).sum())
    wte = np.full((ga.vocab, E), -kappa, np.float32)     # every other token: score -14.5 (< 1.1 x -12.1)
    wte[a_id], wte[b_id] = wa, wb
    sd2 = dict(sd)
    p = "decoder.model.transformer."
    sd2[p + "wte.weight"] = wte
    sd2[p + "ln_f.weight"] = np.zeros(E, np.float32)
    sd2[p + "ln_f.bias"] = beta
    f64 = lambda v: v.astype(np.float64)                  # noqa: E731
    exact = (float(f64(beta) @ f64(wa)), float(f64(beta) @ f64(wb)))
    screen = (float(f64(_bf16(beta)) @ f64(_bf16(wa))), float(f64(_bf16(beta)) @ f64(_bf16(wb))))
    k = float(np.linalg.norm(f64(beta)) * np.linalg.norm(f64(wte), axis=1).max())   # ||h|| max ||w_v||
    return sd2, {"exact": exact, "screen": screen, "hw": k}


class _Round5Bound(HipGPT2Decoder):
    SCREEN_C = 0.0043   # the round-5 constant (2^-8 counted once for both bf16 roundings)


@pytest.mark.parametrize("mode", ["hf", "raw"])
def test_screen_bound_covers_adversarial_near_tie(device, sd, ga, mode):
    """A near-tie whose screen error sits between the round-5 bound and the corrected one: the exact
    f32 winner b is under-rated by the screen by more than the old 2 x bound (so that decoder drops it
    and emits a - the negative control) and by less than the new 2 x bound (the screen keeps b and the
    rescoring picks it).  Under HF greedy (repetition_penalty 1.1) the later steps are near-ties between
    PENALISED NEGATIVE scores (b, a, ... in the history: both scores x 1.1, their errors too), the case
    the runtime's max(rep, 1/rep) factor covers.  Ids must equal the full f32 lm_head's at every step."""
    a_id, b_id = 4000, 9000
    sd2, chk = _adversarial_screen_sd(sd, ga, a_id, b_id)
    (ea, eb), (sa, sb) = chk["exact"], chk["screen"]
    cfg = _cfgs(ga, 0)[mode]
    pf = max(cfg.repetition_penalty, 1.0 / cfg.repetition_penalty)
    gap = sa - sb                          # how far the screen puts b below a (b wins exactly)
    assert 0.0005 < eb - ea < 0.005 and ea < 0 and eb < 0
    assert gap > 2 * 0.0043 * chk["hw"] * 1.001 * pf * 1.05, (gap, chk)           # beyond the old bound
    assert gap < 2 * HipGPT2Decoder.SCREEN_C * chk["hw"] * pf * 0.8, (gap, chk)   # inside the new one
    pre = _prefix(device, 2, ga, 11)
    full = HipGPT2Decoder(sd2, ga, "fp32", device, screen=False)
    scr = HipGPT2Decoder(sd2, ga, "fp32", device)
    old = _Round5Bound(sd2, ga, "fp32", device)
    f, s, o = _ids(full, pre, ga, cfg), _ids(scr, pre, ga, cfg), _ids(old, pre, ga, cfg)
    assert f[0, 0] == b_id, f[0]           # the exact f32 argmax
    assert np.array_equal(s, f), (s, f)
    assert o[0, 0] == a_id, o[0]           # the round-5 constant lost the true argmax here
    if mode == "hf":
        # both tokens in the history by step 2: the near-tie is between penalised negative scores
        assert set(f[0, :2].tolist()) == {a_id, b_id}, f[0]
        assert f[0, 2] in (a_id, b_id)
