"""Beam search / sampling / engine surface on the HIP step-wise decode ABI.

Beam search parity: fp32 HIP forward + vcap/search.py bookkeeping must reproduce the token ids the
reference produced with transformers' beam search (tests/golden: beam3 = preset "precise",
beam4 = preset "detailed")."""
import numpy as np
import pytest
import torch

from helpers import case
from vcap.caption import HipVideoCaptionModel
from vcap.model import HipGPT2Decoder, HipPrefix, HipViTEncoder
from vcap import search

pytestmark = pytest.mark.gpu


def _prefix(name, device):
    meta, g, va, ga, sd, frames = case(name)
    pre = torch.from_numpy(g["inputs_embeds"][:, :4].copy()).to(device)
    dec = HipGPT2Decoder(sd, ga, "fp32", device)
    return meta, g, ga, dec, pre


@pytest.mark.parametrize("name,nb,mx", [("tiny", 3, 24), ("tiny", 4, 40), ("tiny_prompt", 3, 24),
                                        ("b16_b2", 3, 24), ("b16_b2", 4, 40)])
@pytest.mark.parametrize("impl", ["device", "device_eager", "host"])
def test_beam_search_fp32_matches_reference(device, name, nb, mx, impl):
    """Beam ids equal the reference's HF beam search: the device search (csrc/beam.hip, replayed
    graph and eager launches) and the host-bookkeeping restatement."""
    meta, g, ga, dec, pre = _prefix(name, device)
    kw = dict(num_beams=nb, max_new_tokens=mx, min_new_tokens=8, no_repeat_ngram_size=3, repetition_penalty=1.1,
              eos=ga.eos_token_id)
    if impl == "host":
        rows = search.beam_search(dec, pre, meta["prompt_ids"], **kw)
    else:
        rows = search.beam_search_device(dec, pre, meta["prompt_ids"], use_graph=impl == "device", **kw)
    exp = g[f"beam{nb}_ids"]
    assert np.array_equal(np.array(rows, dtype=np.int32), exp), (rows, exp)


def test_step_abi_matches_fused_greedy(device):
    """prefill + step + (identity) reorder reproduce the fused greedy decode's raw logits."""
    meta, g, ga, dec, pre = _prefix("b16_b2", device)
    from vcap.model import GenConfig
    B = meta["B"]
    logits = torch.empty(4, B, ga.vocab, device=device)
    ids = dec.generate_ids(pre, [ga.bos_token_id], GenConfig(4, 0, 0, 1.0, ga.eos_token_id, ga.eos_token_id, False),
                           logits_out=logits)
    st = search._StepState(dec, B, 5, 4)
    l0 = st.prefill(pre, [ga.bos_token_id])
    torch.testing.assert_close(l0, logits[0], rtol=0, atol=1e-5)
    st.reorder(torch.arange(B, device=device), 5)
    l1 = st.step(ids[:, 0], 5)
    torch.testing.assert_close(l1, logits[1], rtol=0, atol=1e-4)


def test_sampling_respects_processors(device):
    meta, g, ga, dec, pre = _prefix("b16_b2", device)
    rows = search.sample(dec, pre, [ga.bos_token_id], temperature=0.9, top_p=0.9, max_new_tokens=24,
                         min_new_tokens=8, no_repeat_ngram_size=3, repetition_penalty=1.05, eos=ga.eos_token_id,
                         seed=3)
    for r in rows:
        assert ga.eos_token_id not in r[:8]
        tri = [tuple(r[i:i + 3]) for i in range(len(r) - 2) if ga.eos_token_id not in r[i:i + 3]]
        assert len(tri) == len(set(tri))
    again = search.sample(dec, pre, [ga.bos_token_id], temperature=0.9, top_p=0.9, max_new_tokens=24,
                          min_new_tokens=8, no_repeat_ngram_size=3, repetition_penalty=1.05, eos=ga.eos_token_id,
                          seed=3)
    assert rows == again


def test_engine_surface_end_to_end(device):
    """core.engine.InferenceEngine.infer_video with id prompts: greedy / beam / sampling candidates."""
    from core.config import InferenceConfig
    from core.engine import InferenceEngine
    meta, g, va, ga, sd, frames = case("tiny")
    cfg = InferenceConfig(vit_name="vit_tiny_test", gpt2_name="gpt2_tiny_test", num_frames=4, precision="fp32",
                          device="cuda:0", weights_seed=1, prompt2="ids:5 900", prompt3="ids:17")
    eng = InferenceEngine(cfg)
    res = eng.infer_video(torch.from_numpy(frames).to(device))
    d = res.to_api_dict()
    assert set(d) == {"S1", "S2", "S3", "BEST"} and d["BEST"]["key"] in {"S1", "S2", "S3"}
    # greedy candidate through the engine == reference greedy ids (clean_text of id strings)
    text = eng._generate_once(torch.from_numpy(frames).to(device), "", num_beams=1, max_new_tokens=24,
                              temperature=1.0, top_p=1.0, no_repeat_ngram_size=3, repetition_penalty=1.1)
    assert isinstance(text, str) and len(text) > 0


def test_caption_model_surface(device):
    meta, g, va, ga, sd, frames = case("b16_b2")
    m = HipVideoCaptionModel(sd, "vit_base_patch16_224", "gpt2", 4, "fp32", device)
    video = torch.from_numpy(frames).to(device)
    emb = m.encoder(video)
    np.testing.assert_allclose(emb.cpu().numpy(), g["encoder_out"], rtol=1e-4, atol=1e-4)
    mapped = m.decoder.mapper(emb)
    assert mapped.shape == (meta["B"], 4 * 768)
    texts = m.decoder.generate(emb.unsqueeze(1), prompt="", max_new_tokens=24, num_beams=1, temperature=1.0,
                               no_repeat_ngram_size=3, repetition_penalty=1.1)
    assert len(texts) == meta["B"]


@pytest.mark.parametrize("nb,mx", [(3, 24), (4, 40)])
def test_beam_search_32_rows_fp32_matches_reference(device, nb, mx):
    """The bench's decode group shape for GPT-2 small (8 sequences x 3 / 4 beams = 24 / 32 rows): the
    beam lm_head streamed with both 16-row halves in one workgroup (vcap_lm_head_lse_kernel, MT = 2) and
    the f32 mlp c_proj on the 8-wave GEMV in two 16-row chunks; 4 copies of the reference's 2 clips give
    the reference's hypotheses for every copy."""
    meta, g, ga, dec, pre = _prefix("b16_b2", device)
    reps = 8 // pre.shape[0]
    rows = search.beam_search_device(dec, pre.repeat(reps, 1, 1).contiguous(), meta["prompt_ids"], num_beams=nb,
                                     max_new_tokens=mx, min_new_tokens=8, no_repeat_ngram_size=3,
                                     repetition_penalty=1.1, eos=ga.eos_token_id)
    exp = g[f"beam{nb}_ids"]
    assert np.array_equal(np.array(rows, dtype=np.int32), np.concatenate([exp] * reps)), rows


@pytest.mark.parametrize("nb,mx", [(3, 24), (4, 40)])
def test_beam_search_bf16_rows_invariant(device, nb, mx):
    """bf16 device beam search: each of 4 copies of 2 sequences (24 / 32 rows: the streamed beam lm_head
    with two row halves per workgroup) finds exactly the hypotheses of the 2 sequences searched alone
    (6 / 8 rows: one row half) - every row's logits and log_softmax partials are computed the same way
    whatever the row count."""
    meta, g, va, ga, sd, frames = case("b16_b2")
    dec = HipGPT2Decoder(sd, ga, "bf16", device)
    pre = torch.from_numpy(g["inputs_embeds"][:, :4].copy()).to(device)
    kw = dict(num_beams=nb, max_new_tokens=mx, min_new_tokens=8, no_repeat_ngram_size=3, repetition_penalty=1.1,
              eos=ga.eos_token_id)
    alone = search.beam_search_device(dec, pre, meta["prompt_ids"], **kw)
    reps = 8 // pre.shape[0]
    many = search.beam_search_device(dec, pre.repeat(reps, 1, 1).contiguous(), meta["prompt_ids"], **kw)
    assert many == alone * reps, (many, alone)


@pytest.mark.parametrize("cap", [48, 96])
def test_beam_search_capped_grids_fp32_matches_reference(device, cap):
    """vcap_beam_params.max_blocks (ABI v14: the pipeline's decode grid cap, now applied to beam searches):
    capped step GEMV grids (wider tiles, no half tiles) and a capped beam lm_head grid (more column tiles
    per workgroup, fewer log_softmax partials) reproduce the reference's beam-3 / beam-4 ids at 8 and 32 rows."""
    meta, g, ga, dec, pre = _prefix("b16_b2", device)
    for nb, mx in ((3, 24), (4, 40)):
        kw = dict(num_beams=nb, max_new_tokens=mx, min_new_tokens=8, no_repeat_ngram_size=3, repetition_penalty=1.1,
                  eos=ga.eos_token_id, max_blocks=cap)
        exp = g[f"beam{nb}_ids"]
        rows = search.beam_search_device(dec, pre, meta["prompt_ids"], **kw)
        assert np.array_equal(np.array(rows, dtype=np.int32), exp), (nb, rows, exp)
        reps = 8 // pre.shape[0]
        rows = search.beam_search_device(dec, pre.repeat(reps, 1, 1).contiguous(), meta["prompt_ids"], **kw)
        assert np.array_equal(np.array(rows, dtype=np.int32), np.concatenate([exp] * reps)), (nb, rows)
