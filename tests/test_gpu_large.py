"""BASELINE configs[3] on the HIP path: 32-frame clips, ViT-L/14 (257 tokens, 16 heads, 24 blocks)
+ GPT-2-medium (E=1024, 24 layers), preset "detailed" (beam 4, max_new 40).

Parity against tests/golden/l14_medium (the reference's own ViTFrameEncoder + InferenceEngine
._generate_once + GPT2TextDecoder.generate run in the build container, make_goldens.py): fp32 mode
encoder within 1e-4, HF-greedy and beam-4 token-identical, step logits within 1e-3."""
import numpy as np
import pytest
import torch

from helpers import case
from vcap import search
from vcap.model import GenConfig, HipGPT2Decoder, HipPrefix, HipViTEncoder, trim_generated

pytestmark = pytest.mark.gpu

_M = {}


def _models(device, prec="fp32"):
    meta, g, va, ga, sd, frames = case("l14_medium")
    if prec not in _M:
        _M.clear()
        _M[prec] = (HipViTEncoder(sd, va, prec, device), HipPrefix(sd, ga.n_embd, device=device),
                    HipGPT2Decoder(sd, ga, prec, device))
    enc, pre, dec = _M[prec]
    return meta, g, va, ga, enc, pre, dec, torch.from_numpy(frames).to(device)


def test_l14_encoder_fp32(device):
    meta, g, va, ga, enc, pre, dec, video = _models(device)
    out, prefix = enc.encode(video, pre)
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy(), g["encoder_out"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(prefix.cpu().numpy(), g["inputs_embeds"][:, :4], rtol=1e-4, atol=1e-5)


def test_medium_greedy_fp32_token_identical_and_logits(device):
    meta, g, va, ga, enc, pre, dec, video = _models(device)
    _, prefix = enc.encode(video, pre)
    B = meta["B"]
    logits = torch.empty(24, B, ga.vocab, device=device)
    cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, False)
    ids = dec.generate_ids(prefix, [ga.bos_token_id], cfg, logits_out=logits)
    got = trim_generated(ids, ga.eos_token_id)
    assert np.array_equal(np.array(got, dtype=np.int32), g["hf_greedy_ids"]), (got, g["hf_greedy_ids"])
    lg = logits.double().cpu().numpy()
    for s in range(3):
        v = np.take_along_axis(lg[s], g[f"hf_greedy_logits_s{s}_top_i"].astype(np.int64), axis=1)
        assert np.abs(v - g[f"hf_greedy_logits_s{s}_top_v"]).max() < 1e-3
    cfg.use_graph = True
    again = trim_generated(dec.generate_ids(prefix, [ga.bos_token_id], cfg), ga.eos_token_id)
    assert again == got


@pytest.mark.parametrize("impl", ["device", "host"])
def test_medium_beam4_fp32_matches_reference(device, impl):
    """preset "detailed" (core/inference.py:10): num_beams 4, max_new_tokens 40 - the device search
    (one hipGraph) and the host-bookkeeping restatement."""
    meta, g, va, ga, enc, pre, dec, video = _models(device)
    prefix = torch.from_numpy(g["inputs_embeds"][:, :4].copy()).to(device)
    fn = search.beam_search_device if impl == "device" else search.beam_search
    rows = fn(dec, prefix, meta["prompt_ids"], num_beams=4, max_new_tokens=40, min_new_tokens=8,
              no_repeat_ngram_size=3, repetition_penalty=1.1, eos=ga.eos_token_id)
    exp = g["beam4_ids"]
    assert np.array_equal(np.array(rows, dtype=np.int32), exp), (rows, exp)


def test_medium_beam4_fp32_32_rows(device):
    """The bench's configs[3] decode shape in fp32 (bench.py --dec-precision fp32: two batches of 4
    videos x 4 beams = 32 decoder rows, whose f32 LayerNorm-prologue tiles take 16-row chunks): the
    reference clips repeated to 8 sequences give the reference's beam-4 hypotheses for every copy."""
    meta, g, va, ga, enc, pre, dec, video = _models(device)
    prefix = torch.from_numpy(g["inputs_embeds"][:, :4].copy()).to(device)
    reps = 8 // prefix.shape[0]
    rows = search.beam_search_device(dec, prefix.repeat(reps, 1, 1).contiguous(), meta["prompt_ids"], num_beams=4,
                                     max_new_tokens=40, min_new_tokens=8, no_repeat_ngram_size=3,
                                     repetition_penalty=1.1, eos=ga.eos_token_id)
    exp = g["beam4_ids"]
    assert np.array_equal(np.array(rows, dtype=np.int32), np.concatenate([exp] * reps)), rows


def test_l14_medium_bf16_close(device):
    """bf16 throughput mode at configs[3] shapes: encoder within 5e-2 abs of the fp32 reference
    (24 blocks of bf16 operand rounding), first greedy token identical where the reference's top-2
    gap exceeds 0.1 (teacher-forced from the reference prefix)."""
    meta, g, va, ga, enc, pre, dec, video = _models(device, "bf16")
    out, _ = enc.encode(video, pre)
    err = np.abs(out.cpu().numpy() - g["encoder_out"]).max()
    assert err < 5e-2, err
    prefix = torch.from_numpy(g["inputs_embeds"][:, :4].copy()).to(device)
    logits = torch.empty(24, meta["B"], ga.vocab, device=device)
    ids = dec.generate_ids(prefix, meta["prompt_ids"], GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id,
                                                                 False), logits_out=logits)
    tv = g["hf_greedy_logits_s0_top_v"]
    got = np.take_along_axis(logits[0].double().cpu().numpy(), g["hf_greedy_logits_s0_top_i"].astype(np.int64), 1)
    assert np.abs(got - tv).max() < 1e-1
    sure = (tv[:, 0] - tv[:, 1]) > 0.1
    assert np.array_equal(ids[:, 0].cpu().numpy()[sure], g["hf_greedy_ids"][sure, 0])


def test_medium_beam4_bf16_rows_invariant(device):
    """bf16 GPT-2-medium beam 4 (configs[3]'s decoder): the reference clips searched alone (one 16-row half
    per lm_head workgroup) and 4 copies of them at 32 rows (both halves in one workgroup,
    vcap_lm_head_lse_kernel<bf16, 8, 4, 2>) give every copy the same hypotheses."""
    meta, g, va, ga, enc, pre, dec, video = _models(device, "bf16")
    prefix = torch.from_numpy(g["inputs_embeds"][:, :4].copy()).to(device)
    kw = dict(num_beams=4, max_new_tokens=40, min_new_tokens=8, no_repeat_ngram_size=3, repetition_penalty=1.1,
              eos=ga.eos_token_id)
    alone = search.beam_search_device(dec, prefix, meta["prompt_ids"], **kw)
    reps = 8 // prefix.shape[0]
    many = search.beam_search_device(dec, prefix.repeat(reps, 1, 1).contiguous(), meta["prompt_ids"], **kw)
    assert many == alone * reps, (many, alone)


def test_medium_beam4_fp32_32_rows_capped(device):
    """The bench's configs[3] fp32 decode as the pipeline runs it: 32 rows with the step grids and the beam
    lm_head capped at 96 workgroups (vcap_beam_params.max_blocks) - the reference's hypotheses per copy."""
    meta, g, va, ga, enc, pre, dec, video = _models(device)
    prefix = torch.from_numpy(g["inputs_embeds"][:, :4].copy()).to(device)
    reps = 8 // prefix.shape[0]
    rows = search.beam_search_device(dec, prefix.repeat(reps, 1, 1).contiguous(), meta["prompt_ids"], num_beams=4,
                                     max_new_tokens=40, min_new_tokens=8, no_repeat_ngram_size=3,
                                     repetition_penalty=1.1, eos=ga.eos_token_id, max_blocks=96)
    assert np.array_equal(np.array(rows, dtype=np.int32), np.concatenate([g["beam4_ids"]] * reps)), rows
