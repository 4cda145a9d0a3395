"""CPU suite: the oracle (oracle/vcap_oracle.py) against the reference's recorded outputs,
the portable PRNG, host-side decode bookkeeping, and the C ABI surface of libvcap_hip.so
(load + every declared symbol; no compute calls without a GPU)."""
import re
from pathlib import Path

import numpy as np
import pytest
import torch

from helpers import case, golden, pad_rows
from oracle import vcap_oracle as O
from vcap import _native as N
from vcap import prng, weights, configs
from vcap.model import raw_greedy_tokens, trim_generated

ROOT = Path(__file__).resolve().parents[1]


def _prefix_inputs(meta, sd, va, ga, frames):
    video = torch.from_numpy(frames)
    with torch.no_grad():
        enc = O.encoder(sd, va, video)
        pre = O.mapper(sd, O.prefix_norm(enc, meta["ln_scale"], meta["in_weight"]), ga.n_embd, 4)
        x = O.build_inputs(sd, ga, pre, meta["prompt_ids"])
    return enc, x


@pytest.mark.parametrize("name", ["tiny", "tiny_prompt"])
def test_oracle_matches_reference_tiny(name):
    meta, g, va, ga, sd, frames = case(name)
    assert weights_digest_ok(sd, meta)
    enc, x = _prefix_inputs(meta, sd, va, ga, frames)
    np.testing.assert_allclose(enc.numpy(), g["encoder_out"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(x.numpy(), g["inputs_embeds"], rtol=1e-5, atol=1e-6)
    with torch.no_grad():
        ids, lg = O.generate_greedy(sd, ga, x, return_logits=True)
        raw = O.generate_raw_greedy(sd, ga, x)
    assert np.array_equal(ids.numpy(), g["hf_greedy_ids"])
    assert np.abs(torch.stack(lg[:3], 1).numpy() - g["hf_greedy_logits"]).max() < 1e-4
    assert np.array_equal(pad_rows(raw, 24), g["raw_greedy_ids"])


@pytest.mark.slow
def test_oracle_matches_reference_b16_b2():
    meta, g, va, ga, sd, frames = case("b16_b2")
    enc, x = _prefix_inputs(meta, sd, va, ga, frames)
    np.testing.assert_allclose(enc.numpy(), g["encoder_out"], rtol=1e-4, atol=1e-5)
    with torch.no_grad():
        ids, lg = O.generate_greedy(sd, ga, x, return_logits=True)
    assert np.array_equal(ids.numpy(), g["hf_greedy_ids"])
    for s in range(3):
        got = np.take_along_axis(lg[s].numpy(), g[f"hf_greedy_logits_s{s}_top_i"].astype(np.int64), 1)
        assert np.abs(got - g[f"hf_greedy_logits_s{s}_top_v"]).max() < 1e-4


def weights_digest_ok(sd, meta):
    import hashlib
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k], dtype=np.float32).tobytes())
    return h.hexdigest() == meta["weights_sha256"]


def test_prng_is_deterministic_and_shaped():
    a = prng.normal(1, "x", (3, 5), 0.02)
    b = prng.normal(1, "x", (3, 5), 0.02)
    c = prng.normal(2, "x", (3, 5), 0.02)
    assert a.dtype == np.float32 and a.shape == (3, 5)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    u = prng.uniform(0, "u", (100000,))
    assert 0.0 <= u.min() and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.01
    z = prng.normal(0, "z", (200000,))
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01


def test_ngram_ban_rule():
    # NoRepeatNGramLogitsProcessor semantics (transformers logits_process.py)
    assert O.banned_ngram_tokens([5, 6, 7, 5, 6], 3) == [7]
    assert O.banned_ngram_tokens([5, 6], 3) == []
    assert O.banned_ngram_tokens([1, 1, 1], 3) == [1]
    assert O.banned_ngram_tokens([4, 4, 4, 4], 2) == [4, 4, 4]


def test_trim_generated_matches_hf_stopping():
    eos = 9
    ids = torch.tensor([[1, 9, 9, 9], [2, 3, 9, 9]], dtype=torch.int32)
    assert trim_generated(ids, eos) == [[1, 9, 9], [2, 3, 9]]
    assert raw_greedy_tokens(ids, eos) == [[1, 9], [2, 3, 9]]
    ids = torch.tensor([[1, 2, 3]], dtype=torch.int32)
    assert trim_generated(ids, eos) == [[1, 2, 3]]


def test_library_exports_every_header_symbol():
    header = (ROOT / "include" / "vcap.h").read_text()
    declared = set(re.findall(r"\b(vcap_[a-z0-9_]+)\s*\(", header))
    assert declared == set(N.SIGNATURES), declared ^ set(N.SIGNATURES)
    lib = N.lib()
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.vcap_abi_version() == N.ABI_VERSION


def test_gemm_mx_argument_checks_without_gpu():
    """vcap_gemm_mx refuses an MXFP8 output whose scale buffer is not 8-byte aligned (the epilogue
    stores 8 scale bytes at once) before touching the device; placeholder pointers are never read."""
    lib = N.lib()
    args = (16, 16, 16, 16, N.DT_MXFP8, 16, 128)
    assert lib.vcap_gemm_mx(*args, 17, 256, 128, 256, 16, 1, None, None) == N.E_ARG
    assert b"8-byte aligned" in lib.vcap_last_error()
    assert lib.vcap_gemm_mx(*args, 16, 256, 128, 256, 16, 0, None, None) == N.E_UNSUPPORTED  # MXFP8 out needs GELU


def test_workspace_queries_without_gpu():
    import ctypes as C
    va, ga = configs.vit_arch("vit_base_patch16_224"), configs.gpt2_arch("gpt2")
    layers = (N.VitLayer * va.depth)()
    d = N.VitDesc(dtype=N.DT_BF16, dim=va.dim, depth=va.depth, heads=va.heads, patch=va.patch, image=va.image,
                  mlp=va.mlp, video_dim=256, kpad=768, ln_eps=1e-6, layers=layers)
    ws = N.lib().vcap_vit_workspace_bytes(C.byref(d), 8, 16)
    M = 8 * 16 * 197
    assert ws >= M * 768 * 4 + M * 3072 * 2
    gl = (N.GPT2Layer * ga.n_layer)()
    gd = N.GPT2Desc(dtype=N.DT_BF16, n_embd=768, n_layer=12, n_head=12, vocab=50257, n_positions=1024, prefix_len=4,
                    ln_eps=1e-5, layers=gl)
    assert N.lib().vcap_gpt2_workspace_bytes(C.byref(gd), 8, 5, 24) > 0
    # rows-packed decoder weights: whole 16-row tiles x K/KS slabs x 1 KiB (csrc/decode.hip)
    assert N.lib().vcap_rows_packed_bytes(N.DT_BF16, 50257, 768) == 3142 * 24 * 1024
    assert N.lib().vcap_rows_packed_bytes(N.DT_F32, 2304, 768) == 144 * 48 * 1024
    assert N.lib().vcap_rows_packed_bytes(N.DT_BF16, 16, 100) == 0
    bad = N.VitDesc(dtype=N.DT_BF16, dim=100, depth=1, heads=1, patch=16, image=224, mlp=400, video_dim=256,
                    kpad=768, ln_eps=1e-6, layers=layers)
    assert N.lib().vcap_vit_workspace_bytes(C.byref(bad), 1, 1) == 0


def test_golden_fixtures_are_self_consistent():
    for name in ("tiny", "tiny_prompt", "b16_b2", "b16_b8"):
        meta, g = golden(name)
        assert g["hf_greedy_ids"].shape[0] == meta["B"]
        assert meta["vit_vs_hf_vitmodel_maxabs"] < 1e-4  # restated timm ViT == transformers.ViTModel


@pytest.mark.slow
def test_oracle_matches_reference_l14_medium():
    """BASELINE configs[3] shapes (ViT-L/14, 257 tokens, GPT-2-medium): the oracle's backbone on
    2 of the 64 recorded frames (CLS rows) and its greedy decode from the recorded prefix."""
    meta, g, va, ga, sd, frames = case("l14_medium")
    assert weights_digest_ok(sd, meta)
    with torch.no_grad():
        f2 = torch.from_numpy(frames.reshape(-1, 3, va.image, va.image)[:2].copy())
        cls = O.vit_forward_features(sd, va, f2)[:, 0, :]
        np.testing.assert_allclose(cls.numpy(), g["cls_tokens"][:2], rtol=1e-4, atol=1e-4)
        x = torch.from_numpy(g["inputs_embeds"].copy())
        ids, lg = O.generate_greedy(sd, ga, x, return_logits=True)
    assert np.array_equal(ids.numpy(), g["hf_greedy_ids"])
    got = np.take_along_axis(lg[0].numpy(), g["hf_greedy_logits_s0_top_i"].astype(np.int64), 1)
    assert np.abs(got - g["hf_greedy_logits_s0_top_v"]).max() < 1e-4


def test_oracle_mx_quantize_properties():
    """MXFP8 restatement: round trip within half an e4m3 step, block max in [128, 256) after
    scaling, zero block -> scale 0, layout round trip."""
    g = np.random.default_rng(0)
    x = (g.standard_normal((300, 512)) * np.exp2(g.integers(-20, 20, (300, 16, 1))).repeat(32, -1).reshape(300, 512))
    x = x.astype(np.float32)
    x[7, 64:96] = 0
    q, s = O.mx_quantize(x)
    d = O.mx_dequantize(q, s)
    assert s[7, 2] == 0 and not d[7, 64:96].any()
    half = np.repeat(np.exp2(s.astype(np.float64) - 127.0) * 8.0, 32, axis=1)
    assert (np.abs(d - x) <= half).all()
    top = np.abs(x).reshape(300, 16, 32).max(-1) * np.exp2(127.0 - s)
    nz = s > 0
    assert ((top[nz] >= 128) & (top[nz] < 256)).all()
    assert np.array_equal(O.mx_unpack_scales(O.mx_pack_scales(s), 300, 512), s)


@pytest.mark.parametrize("hw", [(240, 320), (480, 640), (224, 224), (100, 150), (1080, 1920), (37, 500)])
def test_oracle_pil_resize_matches_pillow(hw):
    """The Resample.c restatement the GPU preprocessing kernel follows is bit-identical to PIL."""
    from PIL import Image
    h, w = hw
    g = np.random.default_rng(h * 7 + w)
    for img in (g.integers(0, 256, (h, w, 3), dtype=np.uint8),
                (np.add.outer(np.arange(h), 3 * np.arange(w))[:, :, None] * np.array([1, 2, 5]) % 256).astype(np.uint8)):
        ref = np.asarray(Image.fromarray(img).resize((224, 224), Image.BILINEAR))
        assert np.array_equal(O.pil_resize_bilinear(img, 224, 224), ref)


@pytest.mark.parametrize("name,nb,mx", [("tiny", 3, 24), ("tiny", 4, 40), ("tiny_prompt", 3, 24)])
def test_oracle_beam_matches_reference(name, nb, mx):
    """The oracle's HF beam-search restatement (presets precise / detailed) reproduces the
    reference's beam ids from the recorded prefix."""
    meta, g, va, ga, sd, frames = case(name)
    x = torch.from_numpy(g["inputs_embeds"].copy())
    with torch.no_grad():
        rows = O.generate_beam(sd, ga, x, num_beams=nb, max_new_tokens=mx)
    assert np.array_equal(np.array(rows, dtype=np.int32), g[f"beam{nb}_ids"])


@pytest.mark.slow
@pytest.mark.parametrize("nb,mx", [(3, 24), (4, 40)])
def test_oracle_beam_matches_reference_b16_b2(nb, mx):
    meta, g, va, ga, sd, frames = case("b16_b2")
    x = torch.from_numpy(g["inputs_embeds"].copy())
    with torch.no_grad():
        rows = O.generate_beam(sd, ga, x, num_beams=nb, max_new_tokens=mx)
    assert np.array_equal(np.array(rows, dtype=np.int32), g[f"beam{nb}_ids"])


@pytest.mark.parametrize("name,nb", [("b16_b2", 3), ("b16_b2", 4), ("l14_medium", 4)])
def test_oracle_hypothesis_scores_match_reference_beam_scores(name, nb):
    """Rescoring the reference's returned beam hypotheses (HF `sequences_scores`, recorded by
    make_goldens.py) with the processed-log-prob / length formula that vcap.fidelity uses to price
    a reduced-precision beam search reproduces the reference's scores."""
    meta, g, va, ga, sd, frames = case(name)
    x = torch.from_numpy(g["inputs_embeds"].copy())
    with torch.no_grad():
        got = O.hypothesis_scores(sd, ga, x, g[f"beam{nb}_ids"].tolist())
    np.testing.assert_allclose(got, g[f"beam{nb}_scores"], rtol=0, atol=2e-5)
