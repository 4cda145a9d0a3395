"""Plugin-hook registry (shape of the reference core/operators/trt_plugin_hooks.py:7-34).

The reference reserved TensorRT plugin names (core/trt/plugins/README.md:3-6); here every fused
HIP entry point of include/vcap.h is registered under a Hip* plugin name so tooling can
enumerate what replaces which torch op."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List


@dataclass(frozen=True)
class PluginHook:
    """`name` -> the reference op it replaces (`reference_op`, file:line under the reference tree or
    its third-party call site) -> the Hip* plugin name and the include/vcap.h symbol that computes
    it.  `torch_path` is the reference TrtPluginHook's field name for the same thing."""
    name: str
    reference_op: str
    plugin_name: str
    abi_symbol: str = ""
    enabled: bool = True

    @property
    def torch_path(self) -> str:
        return self.reference_op


TrtPluginHook = PluginHook  # the reference's class name
_HOOKS: Dict[str, PluginHook] = {}


def register_plugin_hook(hook: PluginHook) -> None:
    _HOOKS[hook.name] = hook


def get_plugin_hook(name: str):
    return _HOOKS.get(name)


def list_plugin_hooks() -> List[PluginHook]:
    return list(_HOOKS.values())


for _h in (
    PluginHook("temporal_mean_pool", "core/operators/cupy_vit_pool.py:127-186 vit_fused_pool_temporal",
               "HipTemporalMeanPool", "vcap_vit_pool_temporal"),
    PluginHook("prefix_projector", "src/models/text_decoder.py:60-74 mapper (core/operators/cupy_linear_mapper.py)",
               "HipPrefixProjector", "vcap_prefix_project"),
    PluginHook("layernorm_scale", "core/engine.py:44-50 layer_norm(emb) * ln_scale * in_weight",
               "HipLayerNormScale", "vcap_prefix_project"),
    PluginHook("linear_mapper", "core/operators/cupy_linear_mapper.py:137-184 CuPyLinearCompat", "HipLinear",
               "vcap_linear_bias"),
    PluginHook("vit_attention", "src/models/video_encoder.py:112-121 timm Attention (fused_attn -> SDPA)",
               "HipViTAttention", "vcap_vit_attention"),
    PluginHook("vit_encoder", "src/models/video_encoder.py:288-326 ViTFrameEncoder.forward", "HipViTEncode",
               "vcap_vit_encode"),
    PluginHook("gpt2_generate", "src/models/text_decoder.py:131-144 generate (greedy)", "HipGPT2Generate",
               "vcap_gpt2_generate"),
    PluginHook("gpt2_beam_search", "src/models/text_decoder.py:131-144 generate (num_beams > 1)",
               "HipGPT2BeamSearch", "vcap_gpt2_beam_search"),
    PluginHook("gpt2_sample", "src/models/text_decoder.py:131-144 generate (do_sample: natural / safe_sample)",
               "HipGPT2Sample", "vcap_gpt2_sample"),
    PluginHook("frame_transform", "core/preprocessing/frame_loader.py:19-49 (torchvision Resize/ToTensor/Normalize)",
               "HipFrameTransform", "vcap_frames_preprocess"),
    PluginHook("vit_linear_fp8", "timm Linear (qkv / proj / fc1 / fc2) in MXFP8 (BASELINE configs[4])",
               "HipMXFP8Linear", "vcap_gemm_mx"),
    PluginHook("vit_layernorm_fp8", "timm LayerNorm feeding an MXFP8 GEMM (BASELINE configs[4])",
               "HipMXFP8LayerNorm", "vcap_layernorm_mx"),
):
    register_plugin_hook(_h)
