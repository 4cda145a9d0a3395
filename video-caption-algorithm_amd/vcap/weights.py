"""Checkpoint key layout and seeded synthetic weights.

Keys are exactly `VideoCaptionModel.state_dict()` of the reference
(SURVEY.md §8b "Weights / ckpt"; src/models/caption_model.py:41-76,
src/models/video_encoder.py:106, src/models/text_decoder.py:216-236):

  encoder.backbone.{cls_token,pos_embed,patch_embed.proj.*,blocks.N.*,norm.*}
  encoder.proj.{weight,bias}
  decoder.model.transformer.{wte,wpe,h.N.*,ln_f}.*   decoder.model.lm_head.weight (tied)
  decoder.mapper.0.{weight,bias}

Synthetic init: linear / pos / cls weights normal(0.02), GPT-2
c_proj scaled by 1/sqrt(2*n_layer), mapper and encoder.proj with torch's Linear
default U(+-1/sqrt(in)).  Biases and LayerNorm affines are randomised too
(small normals around 0 / 1) so every bias and affine path is exercised by the
parity tests.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np

from .configs import VIDEO_DIM, GPT2Arch, ViTArch
from .prng import normal, uniform

StateDict = Dict[str, np.ndarray]


def _ln(seed: int, sd: StateDict, key: str, dim: int) -> None:
    sd[key + ".weight"] = (1.0 + normal(seed, key + ".weight", (dim,), 0.1)).astype(np.float32)
    sd[key + ".bias"] = normal(seed, key + ".bias", (dim,), 0.02)


def _lin(seed: int, sd: StateDict, key: str, out_f: int, in_f: int, std: float = 0.02) -> None:
    sd[key + ".weight"] = normal(seed, key + ".weight", (out_f, in_f), std)
    sd[key + ".bias"] = normal(seed, key + ".bias", (out_f,), 0.02)


def _torch_default_linear(seed: int, sd: StateDict, key: str, out_f: int, in_f: int) -> None:
    bound = 1.0 / math.sqrt(in_f)
    sd[key + ".weight"] = uniform(seed, key + ".weight", (out_f, in_f), -bound, bound)
    sd[key + ".bias"] = uniform(seed, key + ".bias", (out_f,), -bound, bound)


def synthetic_vit(seed: int, arch: ViTArch, video_dim: int = VIDEO_DIM) -> StateDict:
    sd: StateDict = {}
    d, p = arch.dim, "encoder.backbone."
    sd[p + "cls_token"] = normal(seed, p + "cls_token", (1, 1, d), 0.02)
    sd[p + "pos_embed"] = normal(seed, p + "pos_embed", (1, arch.tokens, d), 0.02)
    sd[p + "patch_embed.proj.weight"] = normal(seed, p + "patch_embed.proj.weight",
                                               (d, 3, arch.patch, arch.patch), 0.02)
    sd[p + "patch_embed.proj.bias"] = normal(seed, p + "patch_embed.proj.bias", (d,), 0.02)
    for i in range(arch.depth):
        b = f"{p}blocks.{i}."
        _ln(seed, sd, b + "norm1", d)
        _lin(seed, sd, b + "attn.qkv", 3 * d, d)
        _lin(seed, sd, b + "attn.proj", d, d)
        _ln(seed, sd, b + "norm2", d)
        _lin(seed, sd, b + "mlp.fc1", arch.mlp, d)
        _lin(seed, sd, b + "mlp.fc2", d, arch.mlp)
    _ln(seed, sd, p + "norm", d)
    _torch_default_linear(seed, sd, "encoder.proj", video_dim, d)
    return sd


def synthetic_gpt2(seed: int, arch: GPT2Arch, video_dim: int = VIDEO_DIM, prefix_len: int = 4) -> StateDict:
    sd: StateDict = {}
    e, p = arch.n_embd, "decoder.model.transformer."
    sd[p + "wte.weight"] = normal(seed, p + "wte.weight", (arch.vocab, e), 0.02)
    sd[p + "wpe.weight"] = normal(seed, p + "wpe.weight", (arch.n_positions, e), 0.01)
    proj_std = 0.02 / math.sqrt(2 * arch.n_layer)
    for i in range(arch.n_layer):
        b = f"{p}h.{i}."
        _ln(seed, sd, b + "ln_1", e)
        # HF Conv1D stores weight as [in, out] (x @ W + b)
        sd[b + "attn.c_attn.weight"] = normal(seed, b + "attn.c_attn.weight", (e, 3 * e), 0.02)
        sd[b + "attn.c_attn.bias"] = normal(seed, b + "attn.c_attn.bias", (3 * e,), 0.02)
        sd[b + "attn.c_proj.weight"] = normal(seed, b + "attn.c_proj.weight", (e, e), proj_std)
        sd[b + "attn.c_proj.bias"] = normal(seed, b + "attn.c_proj.bias", (e,), 0.02)
        _ln(seed, sd, b + "ln_2", e)
        sd[b + "mlp.c_fc.weight"] = normal(seed, b + "mlp.c_fc.weight", (e, 4 * e), 0.02)
        sd[b + "mlp.c_fc.bias"] = normal(seed, b + "mlp.c_fc.bias", (4 * e,), 0.02)
        sd[b + "mlp.c_proj.weight"] = normal(seed, b + "mlp.c_proj.weight", (4 * e, e), proj_std)
        sd[b + "mlp.c_proj.bias"] = normal(seed, b + "mlp.c_proj.bias", (e,), 0.02)
    _ln(seed, sd, p + "ln_f", e)
    sd["decoder.model.lm_head.weight"] = sd[p + "wte.weight"]  # tied
    _torch_default_linear(seed, sd, "decoder.mapper.0", e * prefix_len, video_dim)
    return sd


def synthetic_state_dict(seed: int, vit: ViTArch, gpt2: GPT2Arch, prefix_len: int = 4) -> StateDict:
    sd = synthetic_vit(seed, vit)
    sd.update(synthetic_gpt2(seed, gpt2, prefix_len=prefix_len))
    return sd


def normalize_checkpoint(state) -> StateDict:
    """Accept a raw state_dict or {"model_state": ...} (core/models/model_loader.py:74-75)
    and the legacy `vit.*` -> `encoder.backbone.*` remap (tools/debug_chain.py:47-59)."""
    if isinstance(state, dict) and "model_state" in state:
        state = state["model_state"]
    out: StateDict = {}
    for k, v in state.items():
        if k.startswith("vit."):
            k = "encoder.backbone." + k[len("vit."):]
        if hasattr(v, "detach"):
            v = v.detach().float().cpu().numpy()
        out[k] = np.ascontiguousarray(v, dtype=np.float32)
    if "decoder.model.lm_head.weight" not in out and "decoder.model.transformer.wte.weight" in out:
        out["decoder.model.lm_head.weight"] = out["decoder.model.transformer.wte.weight"]
    return out
