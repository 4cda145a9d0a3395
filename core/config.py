"""Engine configuration (field names/defaults of the reference core/config.py:6-72).

Differences, all additive: `backend` defaults to "hip" (the MI355X runtime; the reference's
"torch" eager backend is not shipped - there is no CPU fallback), `precision` selects the
operand dtype of the ViT kernels ("bf16" = the reference's half-precision autocast, "fp32" parity
mode, "fp8" MXFP8 block GEMMs), `decoder_precision` the GPT-2 decoder's ("auto" = fp32 as in the
reference, so the default surface is token-exact; "bf16" the throughput mode), and
`prompt_ids*` let a caller pass pre-tokenised prompts when no GPT-2 BPE vocab is available.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence


@dataclass(frozen=True)
class MemoryConfig:
    max_gpu_mem_mb: int = 3800
    allow_cuda_empty_cache: bool = True
    allow_cpu_fallback: bool = False
    max_concurrent_gpu_tasks: int = 1


@dataclass(frozen=True)
class TensorRTConfig:
    enabled: bool = False
    engine_path: str = ""
    precision: str = "fp16"
    workspace_mb: int = 512
    plugin_namespace: str = "video_caption_plugins"


@dataclass(frozen=True)
class ViTOptimizeConfig:
    """Kept for config compatibility; the HIP backend always runs its fused kernels
    (tanh-GELU epilogue, fused attention, in-place residual), which is what these switches ask for."""
    enable_fp16: bool = False
    enable_attention_fastpath: bool = True
    prefer_channels_last: bool = True
    enable_torch_compile: bool = True
    torch_compile_mode: str = "reduce-overhead"
    enable_mlp_bias_gelu_fusion: bool = True
    enable_residual_layernorm_fusion: bool = True
    enable_inplace_residual_add_fusion: bool = True
    enable_cupy_fused_pool: bool = False
    cupy_pool_force_fp16: bool = True


@dataclass(frozen=True)
class InferenceConfig:
    ckpt: str = ""
    stage: str = "all"
    vit_name: str = "vit_base_patch16_224"
    gpt2_name: str = "gpt2"
    prefix_len: int = 4
    num_frames: int = 8
    image_size: int = 224
    ln_scale: float = 0.6
    in_weight: float = 0.4
    preset1: str = "precise"
    preset2: str = "precise"
    preset3: str = "natural"
    prompt1: str = ""
    prompt2: str = "State the main action in one short sentence:"
    prompt3: str = "Write a short, natural caption:"
    device: str = "cuda"
    backend: str = "hip"
    memory: MemoryConfig = MemoryConfig()
    tensorrt: TensorRTConfig = TensorRTConfig()
    vit_opt: ViTOptimizeConfig = ViTOptimizeConfig()
    use_cupy_prefix_projector: bool = False
    cupy_prefix_force_fp16: bool = True
    # additive fields
    precision: str = "bf16"                 # ViT operands: bf16 (the reference's autocast) | fp32 | fp8
    decoder_precision: str = "auto"         # GPT-2: auto = fp32, the reference's decoder (text_decoder.py:131-144)
    weights_seed: Optional[int] = None      # synthetic random-init weights when no ckpt is given
    tokenizer_dir: str = ""                 # local vocab.json + merges.txt for string prompts
    use_hipgraph: bool = True
    sample_seed: int = 0
