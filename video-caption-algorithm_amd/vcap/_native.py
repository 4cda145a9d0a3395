"""ctypes binding of the C ABI in include/vcap.h (libvcap_hip.so).

The library is the only compute path of the product: there is no torch or CPU fallback.
If the shared object is missing or fails to load, `lib()` raises; callers never route
around it.  The CuPy operators of the reference kept a torch fallback with
`last_backend`/`last_error` bookkeeping (core/operators/cupy_linear_mapper.py:168-184);
here a failing call raises `VcapError` carrying vcap_last_error().
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_LIB_PATH = Path(__file__).resolve().parent / "_lib" / "libvcap_hip.so"
_lib = None

DT_F32, DT_BF16, DT_MXFP8 = 0, 1, 2
ABI_VERSION = 15

vp, i32, i64, f32, sz = C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_size_t
fp = C.POINTER(C.c_float)


E_ARG, E_WORKSPACE, E_UNSUPPORTED = -1000, -1001, -1002


class VcapError(RuntimeError):
    def __init__(self, msg: str, rc: int = 0):
        super().__init__(msg)
        self.rc = rc


class VitLayer(C.Structure):
    _fields_ = [("ln1_g", vp), ("ln1_b", vp), ("qkv_w", vp), ("qkv_b", vp), ("proj_w", vp), ("proj_b", vp),
                ("ln2_g", vp), ("ln2_b", vp), ("fc1_w", vp), ("fc1_b", vp), ("fc2_w", vp), ("fc2_b", vp),
                ("qkv_ws", vp), ("proj_ws", vp), ("fc1_ws", vp), ("fc2_ws", vp)]


class VitDesc(C.Structure):
    _fields_ = [("dtype", i32), ("dim", i32), ("depth", i32), ("heads", i32), ("patch", i32), ("image", i32),
                ("mlp", i32), ("video_dim", i32), ("kpad", i32), ("ln_eps", f32), ("patch_w", vp),
                ("patch_b", vp), ("cls", vp), ("pos", vp), ("norm_g", vp), ("norm_b", vp), ("proj_w", vp),
                ("proj_b", vp), ("layers", C.POINTER(VitLayer))]


class PrefixDesc(C.Structure):
    _fields_ = [("ln_scale", f32), ("in_weight", f32), ("prefix_len", i32), ("n_embd", i32), ("mapper_w", vp),
                ("mapper_b", vp)]


class GPT2Layer(C.Structure):
    _fields_ = [("ln1_g", vp), ("ln1_b", vp), ("attn_w", vp), ("attn_b", vp), ("aproj_w", vp), ("aproj_b", vp),
                ("ln2_g", vp), ("ln2_b", vp), ("fc_w", vp), ("fc_b", vp), ("mproj_w", vp), ("mproj_b", vp)]


class GPT2Desc(C.Structure):
    _fields_ = [("dtype", i32), ("n_embd", i32), ("n_layer", i32), ("n_head", i32), ("vocab", i32),
                ("n_positions", i32), ("prefix_len", i32), ("ln_eps", f32), ("wte", vp), ("lm_head", vp), ("wpe", vp),
                ("lnf_g", vp), ("lnf_b", vp), ("layers", C.POINTER(GPT2Layer)), ("lm_head_screen", vp),
                ("screen_bound", f32)]


class GenParams(C.Structure):
    _fields_ = [("max_new_tokens", i32), ("min_new_tokens", i32), ("no_repeat_ngram_size", i32),
                ("repetition_penalty", f32), ("eos_token_id", i32), ("pad_token_id", i32), ("use_graph", i32),
                ("max_blocks", i32)]


class BeamParams(C.Structure):
    _fields_ = [("num_beams", i32), ("max_new_tokens", i32), ("min_new_tokens", i32),
                ("no_repeat_ngram_size", i32), ("repetition_penalty", f32), ("length_penalty", f32),
                ("early_stopping", i32), ("eos_token_id", i32), ("use_graph", i32), ("max_blocks", i32)]


class SampleParams(C.Structure):
    _fields_ = [("temperature", f32), ("top_k", i32), ("top_p", C.c_double), ("seed", C.c_uint64)]


# name -> (restype, argtypes); every symbol include/vcap.h declares
SIGNATURES = {
    "vcap_last_error": (C.c_char_p, []),
    "vcap_abi_version": (i32, []),
    "vcap_set_gemm_policy": (i32, [i32]),
    "vcap_stream_create_cu_reserved": (i32, [i32, C.POINTER(C.c_void_p)]),
    "vcap_stream_create_cu_mask": (i32, [C.POINTER(C.c_uint32), i32, C.POINTER(C.c_void_p)]),
    "vcap_stream_destroy": (i32, [vp]),
    "vcap_linear_bias": (i32, [i32, vp, vp, vp, vp, i32, i32, i32, vp]),
    "vcap_gemm": (i32, [i32, i32, vp, i64, vp, i64, vp, i64, i32, i32, i32, vp, i32, vp, i64, i32, i32, i32, i32,
                        i32, vp]),
    "vcap_layernorm": (i32, [i32, vp, i64, vp, i64, vp, vp, i32, i32, f32, vp]),
    "vcap_vit_attention": (i32, [i32, vp, vp, i32, i32, i32, vp]),
    "vcap_vit_qkv_attention": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, vp]),
    "vcap_frames_workspace_bytes": (sz, [i32, i32, i32, i32, i32]),
    "vcap_frames_preprocess": (i32, [vp, i32, i32, i32, i32, i32, fp, fp, vp, vp, vp, sz, vp]),
    "vcap_jpeg_probe": (i32, [vp, sz, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "vcap_jpeg_workspace_bytes": (sz, [vp, sz, i32]),
    "vcap_jpeg_decode_batch": (i32, [C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), i32, vp, vp, sz, vp]),
    "vcap_mx_scale_bytes": (sz, [i32, i32]),
    "vcap_vit_attention_mx": (i32, [vp, vp, vp, i32, i32, i32, vp]),
    "vcap_mx_quantize": (i32, [i32, vp, i64, i32, i32, vp, vp, vp]),
    "vcap_layernorm_mx": (i32, [vp, i64, vp, vp, vp, vp, i32, i32, f32, vp]),
    "vcap_gemm_mx": (i32, [vp, vp, vp, vp, i32, vp, i64, vp, i32, i32, i32, vp, i32, vp, vp]),
    "vcap_vit_pool_temporal": (i32, [i32, vp, vp, i32, i32, i32, i32, i32, vp]),
    "vcap_prefix_project": (i32, [vp, i32, i32, C.POINTER(PrefixDesc), vp, vp]),
    "vcap_rows_packed_bytes": (sz, [i32, i32, i32]),
    "vcap_rows_pack": (i32, [i32, vp, i64, i32, i32, vp, vp]),
    "vcap_vit_workspace_bytes": (sz, [C.POINTER(VitDesc), i32, i32]),
    "vcap_vit_encode": (i32, [C.POINTER(VitDesc), C.POINTER(PrefixDesc), vp, i32, i32, vp, vp, vp, sz, vp]),
    "vcap_vit_layer_fuses_qkv_attention": (i32, [C.POINTER(VitDesc), i32]),
    "vcap_gpt2_workspace_bytes": (sz, [C.POINTER(GPT2Desc), i32, i32, i32]),
    "vcap_gpt2_generate": (i32, [C.POINTER(GPT2Desc), C.POINTER(GenParams), vp, C.POINTER(C.c_int), i32, i32, vp,
                                 vp, vp, sz, vp]),
    "vcap_gpt2_sample": (i32, [C.POINTER(GPT2Desc), C.POINTER(GenParams), C.POINTER(SampleParams), vp,
                               C.POINTER(C.c_int), i32, i32, vp, vp, vp, vp, vp, sz, vp]),
    "vcap_graph_cache_clear": (None, []),
    "vcap_graph_cache_size": (i32, []),
    "vcap_gpt2_max_rows": (i32, []),
    "vcap_gpt2_beam_search_workspace_bytes": (sz, [C.POINTER(GPT2Desc), i32, i32, i32, i32]),
    "vcap_gpt2_beam_search": (i32, [C.POINTER(GPT2Desc), C.POINTER(BeamParams), vp, C.POINTER(C.c_int), i32, i32,
                                    vp, vp, vp, sz, vp]),
    "vcap_decode_attention": (i32, [i32, vp, vp, vp, vp, i32, vp, i32, i32, i32, i32, vp]),
    "vcap_gpt2_beam_workspace_bytes": (sz, [C.POINTER(GPT2Desc), i32, i32, i32]),
    "vcap_gpt2_prefill": (i32, [C.POINTER(GPT2Desc), vp, C.POINTER(C.c_int), i32, i32, i32, i32, vp, vp, sz, vp]),
    "vcap_gpt2_step": (i32, [C.POINTER(GPT2Desc), vp, i32, i32, i32, i32, vp, vp, sz, vp]),
    "vcap_gpt2_reorder": (i32, [C.POINTER(GPT2Desc), vp, i32, i32, i32, i32, vp, sz, vp]),
    "vcap_gpt2_forward_embeds": (i32, [C.POINTER(GPT2Desc), vp, i32, i32, i32, i32, i32, vp, vp, sz, vp]),
    "vcap_probe_enable": (i32, [C.c_char_p, i32]),
    "vcap_probe_read": (i32, [C.c_char_p, fp, C.POINTER(C.c_int)]),
    "vcap_probe_read_launches": (i32, [C.c_char_p, fp, C.POINTER(C.c_int), i32, C.POINTER(C.c_int)]),
}


def library_path() -> Path:
    return Path(os.environ.get("VCAP_LIB", str(_LIB_PATH)))


def lib():
    """Load libvcap_hip.so once; raise if it is absent (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not path.exists():
        raise VcapError(f"libvcap_hip.so not built at {path}; run `python -m vcap.build` "
                        "(or __graft_entry__.build()) - the HIP path has no CPU fallback")
    h = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(h, name)
        fn.restype = res
        fn.argtypes = args
    if h.vcap_abi_version() != ABI_VERSION:
        raise VcapError(f"ABI mismatch: library {h.vcap_abi_version()} vs binding {ABI_VERSION}")
    _lib = h
    return h


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().vcap_last_error()
        raise VcapError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}", rc)


def ptr(t) -> int:
    """Raw device address of a torch tensor (None -> NULL)."""
    return 0 if t is None else t.data_ptr()
