"""Plugin-hook registry (shape of the reference core/operators/trt_plugin_hooks.py:7-34).

The reference reserved TensorRT plugin names (core/trt/plugins/README.md:3-6); here every fused
HIP entry point of include/vcap.h is registered under a Hip* plugin name so tooling can
enumerate what replaces which torch op."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List


@dataclass(frozen=True)
class PluginHook:
    name: str
    torch_path: str
    plugin_name: str
    abi_symbol: str = ""
    enabled: bool = True


TrtPluginHook = PluginHook  # the reference's class name
_HOOKS: Dict[str, PluginHook] = {}


def register_plugin_hook(hook: PluginHook) -> None:
    _HOOKS[hook.name] = hook


def get_plugin_hook(name: str):
    return _HOOKS.get(name)


def list_plugin_hooks() -> List[PluginHook]:
    return list(_HOOKS.values())


for _h in (
    PluginHook("temporal_mean_pool", "core.operators.temporal_pool.TemporalMeanPool", "HipTemporalMeanPool",
               "vcap_vit_pool_temporal"),
    PluginHook("prefix_projector", "core.operators.prefix_projector.PrefixProjector", "HipPrefixProjector",
               "vcap_prefix_project"),
    PluginHook("layernorm_scale", "core.operators.normalization.apply_prefix_norm", "HipLayerNormScale",
               "vcap_prefix_project"),
    PluginHook("linear_mapper", "core.operators.cupy_linear_mapper.CuPyLinearCompat", "HipLinear",
               "vcap_linear_bias"),
    PluginHook("vit_attention", "timm.models.vision_transformer.Attention", "HipViTAttention",
               "vcap_vit_attention"),
    PluginHook("vit_encoder", "src.models.video_encoder.ViTFrameEncoder", "HipViTEncode", "vcap_vit_encode"),
    PluginHook("gpt2_generate", "src.models.text_decoder.GPT2TextDecoder.generate", "HipGPT2Generate",
               "vcap_gpt2_generate"),
    PluginHook("frame_transform", "core.preprocessing.frame_loader (torchvision Resize/ToTensor/Normalize)",
               "HipFrameTransform", "vcap_frames_preprocess"),
    PluginHook("vit_linear_fp8", "timm Linear (qkv / proj / fc1 / fc2) in MXFP8", "HipMXFP8Linear", "vcap_gemm_mx"),
    PluginHook("vit_layernorm_fp8", "timm LayerNorm feeding an MXFP8 GEMM", "HipMXFP8LayerNorm",
               "vcap_layernorm_mx"),
):
    register_plugin_hook(_h)
