"""Architecture constants for the encoder/decoder pairs the hot path serves.

Names follow the reference's `vit_name` / `gpt2_name` config fields
(core/config.py:52-53, backend_config.py:15-16).  The tiny pair keeps
head_dim = 64 (the kernels' specialisation) so the same HIP path is exercised
by the small golden fixtures.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class ViTArch:
    name: str
    dim: int
    depth: int
    heads: int
    patch: int
    image: int = 224
    mlp_ratio: int = 4
    ln_eps: float = 1e-6  # timm ViT LayerNorm eps (video_encoder.py:70-75 -> timm defaults)

    @property
    def head_dim(self) -> int:
        return self.dim // self.heads

    @property
    def grid(self) -> int:
        return self.image // self.patch

    @property
    def num_patches(self) -> int:
        return self.grid * self.grid

    @property
    def tokens(self) -> int:
        return self.num_patches + 1

    @property
    def mlp(self) -> int:
        return self.dim * self.mlp_ratio

    @property
    def patch_k(self) -> int:
        return 3 * self.patch * self.patch

    def flops_per_frame(self, cls_tail: bool = False) -> float:
        """Algorithmic FLOPs per frame (full reference semantics).  cls_tail: the last
        block computed for the class-token row only after its QKV projection (the rows the encoder
        output depends on; what vcap_vit_encode runs)."""
        n, d, m = self.tokens, self.dim, self.mlp
        per_block = 2 * n * d * 3 * d + 2 * 2 * n * n * d + 2 * n * d * d + 2 * 2 * n * d * m
        total = per_block * self.depth + 2 * self.num_patches * self.patch_k * d
        if cls_tail:
            tail = 2 * n * d * 3 * d + 2 * 2 * n * d + 2 * d * d + 2 * 2 * d * m
            total += tail - per_block
        return float(total)


@dataclass(frozen=True)
class GPT2Arch:
    name: str
    n_embd: int
    n_layer: int
    n_head: int
    vocab: int = 50257
    n_positions: int = 1024
    ln_eps: float = 1e-5  # GPT2Config.layer_norm_epsilon default
    bos_token_id: int = 50256
    eos_token_id: int = 50256

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head

    def weight_elems_per_step(self) -> int:
        e = self.n_embd
        return self.n_layer * (e * 3 * e + e * e + 2 * e * 4 * e) + self.vocab * e


VITS = {
    "vit_base_patch16_224": ViTArch("vit_base_patch16_224", 768, 12, 12, 16),
    "vit_large_patch14_224": ViTArch("vit_large_patch14_224", 1024, 24, 16, 14),
    "vit_tiny_test": ViTArch("vit_tiny_test", 128, 2, 2, 16),
}

GPT2S = {
    "gpt2": GPT2Arch("gpt2", 768, 12, 12),
    "gpt2-medium": GPT2Arch("gpt2-medium", 1024, 24, 16),
    "gpt2_tiny_test": GPT2Arch("gpt2_tiny_test", 128, 2, 2, vocab=1024, n_positions=64,
                               bos_token_id=1023, eos_token_id=1023),
}

VIDEO_DIM = 256  # caption_model.py:21 video_dim / encoder out_dim


def vit_arch(name: str) -> ViTArch:
    if name not in VITS:
        raise ValueError(f"Unsupported ViT: {name} (known: {sorted(VITS)})")
    return VITS[name]


def gpt2_arch(name: str) -> GPT2Arch:
    if name not in GPT2S:
        raise ValueError(f"Unsupported GPT-2: {name} (known: {sorted(GPT2S)})")
    return GPT2S[name]
