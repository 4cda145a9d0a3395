"""Engine-level parity: the drop-in surface (core.engine.InferenceEngine, VideoCaptionModel.generate,
the sampling presets) against outputs recorded by running the reference's own engine
(tests/golden/make_goldens.py `surface_case`: core/engine.py:39-83, src/models/caption_model.py:93-101,
HF generate's processed sampling scores).  fp32 mode (the token-exact one)."""
import numpy as np
import pytest
import torch

from helpers import case, golden
from vcap import _native as N
from vcap import search
from vcap.model import trim_generated

pytestmark = pytest.mark.gpu

GREEDY = dict(num_beams=1, max_new_tokens=24, temperature=1.0, top_p=1.0, no_repeat_ngram_size=3,
              repetition_penalty=1.1)
_ENG = {}


def _engine(name, device):
    from core.config import InferenceConfig
    from core.engine import InferenceEngine
    meta, g, va, ga, sd, frames = case(name)
    surf = meta["surface"]
    if name not in _ENG:
        _ENG.clear()
        cfg = InferenceConfig(vit_name=meta["vit"], gpt2_name=meta["gpt2"], num_frames=meta["T"], precision="fp32",
                              device=str(device), weights_seed=meta["weights_seed"], preset1="precise",
                              preset2="precise", preset3="natural", prompt1="", prompt2=surf["prompt_text"],
                              prompt3=surf["prompt_text"])
        _ENG[name] = InferenceEngine(cfg)
    return meta, g, ga, surf, _ENG[name], torch.from_numpy(frames).to(device)


@pytest.mark.parametrize("name", ["tiny", "b16_b2"])
def test_generate_once_greedy_and_precise(device, name):
    """_generate_once strings (decode -> batch_decode -> clean_text) and the ids behind them."""
    from core.inference import preset_to_kwargs
    meta, g, ga, surf, eng, video = _engine(name, device)
    assert eng._generate_once(video, "", **GREEDY) == surf["greedy_text"]
    assert eng._generate_once(video, "", **preset_to_kwargs("precise")) == surf["precise_text"]
    assert eng._generate_once(video, surf["prompt_text"], **GREEDY) == surf["prompt_greedy_text"]
    dec, prefix = eng.model.decoder, eng._prefix(video)
    bos = [ga.bos_token_id]
    assert dec.generate_from_prefix(prefix, bos, **GREEDY, min_new_tokens=8) == g["hf_greedy_ids"].tolist()
    assert dec.generate_from_prefix(prefix, bos, **preset_to_kwargs("precise"), min_new_tokens=8) == surf["precise_ids"]
    pids = dec.tokenizer.encode_prompt(surf["prompt_text"])
    assert dec.generate_from_prefix(prefix, pids, **GREEDY, min_new_tokens=8) == surf["prompt_greedy_ids"]
    assert dec.generate_from_prefix(prefix, pids, **preset_to_kwargs("precise"), min_new_tokens=8) == \
        surf["prompt_precise_ids"]


@pytest.mark.parametrize("name", ["tiny", "b16_b2"])
def test_infer_candidates_s1_s2(device, name):
    """infer() (core/engine.py:66-83): S1 = precise + prompt1, S2 = precise + prompt2 equal the
    reference engine's strings (S3 samples: its parity is the distributional test below)."""
    meta, g, ga, surf, eng, video = _engine(name, device)
    res = eng.infer_video(video)
    assert res.candidates.s1 == surf["precise_text"]
    assert res.candidates.s2 == surf["prompt_precise_text"]
    assert res.best_key in {"S1", "S2", "S3"}


@pytest.mark.parametrize("name", ["tiny", "b16_b2"])
def test_video_caption_model_generate_no_ln_scale(device, name):
    """VideoCaptionModel.generate: encoder -> proj -> decoder.generate WITHOUT the engine's LN-scale
    (src/models/caption_model.py:93-101): every row's text equals the reference's."""
    meta, g, ga, surf, eng, video = _engine(name, device)
    texts = eng.model.generate(video, prompt="", **GREEDY)
    assert texts == surf["model_generate_texts"]


def test_repeated_generate_once_reuses_one_graph(device):
    """50 engine calls with fresh prefix tensors each time: the decode graph cache stays at one
    entry per shape (persistent decode buffers + bounded LRU)."""
    meta, g, ga, surf, eng, video = _engine("tiny", device)
    N.lib().vcap_graph_cache_clear()
    for _ in range(50):
        eng._generate_once(video, "", **GREEDY)
    torch.cuda.synchronize()
    assert N.lib().vcap_graph_cache_size() == 1


@pytest.mark.parametrize("preset", ["natural", "safe_sample"])
def test_device_sampling_warped_scores_match_hf_every_step(device, preset):
    """The distribution `natural` / `safe_sample` draw from, computed by the device sampling path
    (lm_head processor epilogue + csrc/sample.hip warpers inside the decode graph), replaying the
    reference's own sampled history (force_ids): at every step the warped scores (warped_out) equal
    HF's processed scores (same -inf mask, finite scores within 1e-4) and the raw logits equal the
    reference's (tests/golden/tiny, make_goldens.py surface_case)."""
    from vcap.model import GenConfig, HipGPT2Decoder
    meta, g, va, ga, sd, frames = case("tiny")
    kw = meta[preset]
    logits = torch.from_numpy(g[f"{preset}_logits"]).to(device)    # [steps, B, V]
    scores = torch.from_numpy(g[f"{preset}_scores"]).to(device)
    ids = g[f"{preset}_ids"].astype(np.int64)
    steps, B = logits.shape[0], logits.shape[1]
    L = kw["max_new_tokens"]
    force = np.full((B, L), ga.eos_token_id, np.int64)
    force[:, :ids.shape[1]] = ids
    dec = HipGPT2Decoder(sd, ga, "fp32", device)
    cfg = GenConfig(L, kw["min_new_tokens"], kw["no_repeat_ngram_size"], kw["repetition_penalty"], ga.eos_token_id,
                    ga.eos_token_id, True, temperature=kw["temperature"], top_p=kw["top_p"], seed=5)
    prefix = torch.from_numpy(g["inputs_embeds"][:, :4].copy()).to(device)
    warped = torch.empty(L, B, ga.vocab, device=device)
    raw = torch.empty(L, B, ga.vocab, device=device)
    out = dec.generate_ids(prefix, [ga.bos_token_id], cfg, logits_out=raw, warped_out=warped,
                           force_ids=torch.from_numpy(force))
    assert np.array_equal(out.cpu().numpy()[:, :ids.shape[1]], ids)
    for s in range(steps):
        torch.testing.assert_close(raw[s], logits[s], rtol=0, atol=1e-4)
        fin = torch.isfinite(scores[s])
        assert torch.equal(torch.isfinite(warped[s]), fin), s
        torch.testing.assert_close(warped[s][fin], scores[s][fin], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("preset", ["natural", "safe_sample"])
def test_device_sampling_gpt2_vocab_matches_hf_every_step(device, preset):
    """The same check at the full GPT-2 vocab (50,257 columns: the `vcap_sample_kernel<50>` instance
    every `infer()` S3 candidate runs): replaying the reference engine's sampled history
    (tests/golden/b16_b2_sample, make_goldens.py `sample_case`), at every step and row the device's
    finite warped scores are exactly HF's TopK(50) -> TopP support (same token set) with values within
    1e-4, and the raw logits match the reference's top-64 within 1e-3 (core/inference.py:12-15,
    src/models/text_decoder.py:137-139)."""
    from vcap.model import GenConfig, HipGPT2Decoder
    meta, g, va, ga, sd, frames = case("b16_b2_sample")
    kw = meta[preset]
    ids = g[f"{preset}_ids"].astype(np.int64)
    wi, wv = g[f"{preset}_warped_idx"], g[f"{preset}_warped_val"]
    top_i, top_v = g[f"{preset}_top_i"], g[f"{preset}_top_v"]
    steps, B, V = wi.shape[0], wi.shape[1], ga.vocab
    assert V == 50257
    L = kw["max_new_tokens"]
    force = np.full((B, L), ga.eos_token_id, np.int64)
    force[:, :ids.shape[1]] = ids
    dec = HipGPT2Decoder(sd, ga, "fp32", device)
    cfg = GenConfig(L, kw["min_new_tokens"], kw["no_repeat_ngram_size"], kw["repetition_penalty"], ga.eos_token_id,
                    ga.eos_token_id, True, temperature=kw["temperature"], top_p=kw["top_p"], seed=11)
    prefix = torch.from_numpy(g["inputs_embeds"][:, :4].copy()).to(device)
    warped = torch.empty(L, B, V, device=device)
    raw = torch.empty(L, B, V, device=device)
    out = dec.generate_ids(prefix, [ga.bos_token_id], cfg, logits_out=raw, warped_out=warped,
                           force_ids=torch.from_numpy(force))
    assert np.array_equal(out.cpu().numpy()[:, :ids.shape[1]], ids)
    warped, raw = warped.cpu().numpy(), raw.cpu().numpy()
    for s in range(steps):
        for b in range(B):
            np.testing.assert_allclose(raw[s, b, top_i[s, b]], top_v[s, b], rtol=0, atol=1e-3)
            keep = wi[s, b] >= 0
            fin = np.flatnonzero(np.isfinite(warped[s, b]))
            assert np.array_equal(fin, np.sort(wi[s, b][keep])), (s, b)
            np.testing.assert_allclose(warped[s, b, wi[s, b][keep]], wv[s, b][keep], rtol=1e-5, atol=1e-4)


def test_device_sampling_draws_follow_the_warped_distribution(device):
    """3200 first-token draws (100 rows x 32 seeds) of one prefix: every draw lies in the warped
    support, and the draw frequencies match softmax(warped scores) (chi-square, pooled bins)."""
    from scipy import stats
    from vcap.model import GenConfig, HipGPT2Decoder
    meta, g, va, ga, sd, frames = case("tiny")
    dec = HipGPT2Decoder(sd, ga, "fp32", device)
    rows = 100
    prefix = torch.from_numpy(np.repeat(g["inputs_embeds"][:1, :4], rows, axis=0).copy()).to(device)
    counts = np.zeros(ga.vocab)
    probs = None
    for seed in range(32):
        cfg = GenConfig(1, 0, 3, 1.05, ga.eos_token_id, ga.eos_token_id, True, temperature=0.9, top_p=0.9, seed=seed)
        warped = torch.empty(1, rows, ga.vocab, device=device)
        ids = dec.generate_ids(prefix, [ga.bos_token_id], cfg, warped_out=warped).cpu().numpy()[:, 0]
        p = torch.softmax(warped[0, 0].double(), -1).cpu().numpy()
        assert probs is None or np.allclose(p, probs)
        probs = p
        assert np.all(p[ids] > 0), "a draw outside the warped support"
        np.add.at(counts, ids, 1)
    n = counts.sum()
    order = np.argsort(-probs)
    big = [i for i in order if probs[i] * n >= 5]
    f_obs = np.append(counts[big], n - counts[big].sum())
    f_exp = np.append(probs[big] * n, n - probs[big].sum() * n)
    keep = f_exp > 0
    p_value = stats.chisquare(f_obs[keep], f_exp[keep]).pvalue
    print(f"chi-square over {keep.sum()} bins: p = {p_value:.3g}")
    assert p_value > 1e-4


def test_checkpoint_roundtrip(device, tmp_path):
    """A reference-format checkpoint ({"model_state": state_dict}, src/cli/train_caption_mapper.py:301-305)
    loaded through load_caption_model(ckpt=...) (model_loader.py:31-80) decodes the golden ids;
    keys missing from the checkpoint follow the reference's strict=False (logged, kept at init)."""
    from core.config import InferenceConfig
    from core.models.model_loader import load_caption_model
    meta, g, va, ga, sd, frames = case("tiny")
    ck = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}
    path = tmp_path / "ckpt.pt"
    torch.save({"model_state": ck, "step": 1, "epoch": 0}, path)
    cfg = InferenceConfig(ckpt=str(path), vit_name=meta["vit"], gpt2_name=meta["gpt2"], num_frames=meta["T"],
                          precision="fp32", device=str(device), weights_seed=meta["weights_seed"])
    m = load_caption_model(cfg)
    ids = m.generate_ids(torch.from_numpy(frames).to(device), [ga.bos_token_id])
    assert trim_generated(ids, ga.eos_token_id) == g["hf_greedy_ids"].tolist()
    # strict=False: drop a key -> it keeps the initialiser's value (seeded init = the same weights here)
    ck2 = dict(ck)
    ck2.pop("encoder.proj.bias")
    torch.save(ck2, path)
    m2 = load_caption_model(cfg)
    ids2 = m2.generate_ids(torch.from_numpy(frames).to(device), [ga.bos_token_id])
    assert torch.equal(ids2, ids)


def test_default_config_decodes_in_fp32(device):
    """InferenceEngine(InferenceConfig()) - the drop-in default - runs the reference's precision split:
    ViT in bf16 (the reference's half-precision autocast, src/models/video_encoder.py:261-264) and the
    GPT-2 decoder in fp32 (text_decoder.py:131-144), so its greedy captions are those of an fp32
    decoder (here: the full f32 lm_head on the same prefix) and, on the b16_b2 golden clips, the
    reference's own greedy ids."""
    from core.config import InferenceConfig
    from core.engine import InferenceEngine
    from vcap.model import GenConfig, HipGPT2Decoder
    meta, g, va, ga, sd, frames = case("b16_b2")
    cfg = InferenceConfig(device=str(device), num_frames=meta["T"], weights_seed=meta["weights_seed"])
    assert (cfg.precision, cfg.decoder_precision) == ("bf16", "auto")
    eng = InferenceEngine(cfg)
    assert eng.model.hip_encoder.precision == "bf16"
    assert eng.model.decoder_precision == "fp32"
    hip = eng.model.decoder.hip
    assert hip.precision == "fp32" and hip.dt == N.DT_F32 and hip.screen
    video = torch.from_numpy(frames).to(device)
    prefix = eng._prefix(video)
    bos = [ga.bos_token_id]
    got = eng.model.decoder.generate_from_prefix(prefix, bos, **GREEDY, min_new_tokens=8)
    full = HipGPT2Decoder(sd, ga, "fp32", device, screen=False)
    gc = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
    assert got == trim_generated(full.generate_ids(prefix, bos, gc), ga.eos_token_id)
    assert got == g["hf_greedy_ids"].tolist()
    # bf16 is still selectable (the throughput mode of the bench line)
    eng16 = InferenceEngine(InferenceConfig(device=str(device), num_frames=meta["T"],
                                            weights_seed=meta["weights_seed"], decoder_precision="bf16"))
    assert eng16.model.decoder.hip.precision == "bf16"
