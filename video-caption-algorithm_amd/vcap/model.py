"""Device-resident ViT encoder and GPT-2 decoder driven through the C ABI.

`HipViTEncoder` and `HipGPT2Decoder` own the packed weights in HBM (operand dtype bf16 for
throughput or fp32 for the parity mode), build the include/vcap.h descriptors once, keep a
reusable workspace, and issue one ABI call per encode / per whole decode.

Weight packing from the reference's state-dict layout:
  * ViT Linear weights keep torch's [out, in] layout (K contiguous), the patch-embed conv
    weight is flattened to [D, 3*p*p] and zero-padded in K to the GEMM K step;
  * GPT-2 Conv1D weights ([in, out], x @ W + b) are transposed to [out, in];
  * wte is shared by the embedding lookup and the tied lm_head (text_decoder.py:28);
  * LayerNorm affines, biases, positional tables, encoder.proj and the mapper stay fp32.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _native as N
from .configs import VIDEO_DIM, GPT2Arch, ViTArch

_DTYPES = {"bf16": (N.DT_BF16, torch.bfloat16), "fp32": (N.DT_F32, torch.float32)}
# ViT only: "fp8" = MXFP8 block GEMMs (QKV / attn-proj / fc1 / fc2: e4m3 + E8M0 per 32 K elements,
# the gfx950 scaled-MFMA format; BASELINE configs[4]); patch-embed and QK^T / PV run in bf16.
_VIT_DTYPES = dict(_DTYPES, fp8=(N.DT_MXFP8, torch.bfloat16))


def _dtype(mode: str):
    if mode not in _DTYPES:
        raise ValueError(f"precision must be one of {sorted(_DTYPES)}, got {mode!r}")
    return _DTYPES[mode]


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class _Workspace:
    def __init__(self, device):
        self.device = device
        self.buf: Optional[torch.Tensor] = None

    def get(self, nbytes: int) -> torch.Tensor:
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        return self.buf


class HipViTEncoder:
    """ViTFrameEncoder.forward (src/models/video_encoder.py:288-326) on the HIP path."""

    MX_GEMMS = ("qkv", "proj", "fc1", "fc2")

    def __init__(self, sd: Dict[str, np.ndarray], arch: ViTArch, precision: str = "bf16", device="cuda",
                 video_dim: int = VIDEO_DIM, mx_gemms: Sequence[str] = MX_GEMMS):
        """precision "fp8": the block GEMMs named in `mx_gemms` run in MXFP8, the others in bf16
        (their weights bf16, their scales NULL in the descriptor: csrc/runtime.hip picks per GEMM)."""
        N.lib()
        self.arch, self.precision, self.device = arch, precision, torch.device(device)
        if precision not in _VIT_DTYPES:
            raise ValueError(f"precision must be one of {sorted(_VIT_DTYPES)}, got {precision!r}")
        bad = set(mx_gemms) - set(self.MX_GEMMS)
        if bad:
            raise ValueError(f"mx_gemms: unknown GEMM(s) {sorted(bad)}; choose from {self.MX_GEMMS}")
        self.dt, tdt = _VIT_DTYPES[precision]
        mx = self.dt == N.DT_MXFP8
        self.mx_gemms = tuple(g for g in self.MX_GEMMS if g in mx_gemms) if mx else ()
        self.video_dim = video_dim
        p = "encoder.backbone."
        dev = self.device

        def f32(k, shape=None):
            t = torch.from_numpy(np.ascontiguousarray(sd[k], dtype=np.float32))
            if shape is not None:
                t = t.reshape(shape)
            return t.to(dev).contiguous()

        def wt(k, shape=None):
            return f32(k, shape).to(tdt).contiguous()

        def wmx(k):
            """-> (e4m3 [N, K] uint8, E8M0 scales) through vcap_mx_quantize (kept alive in _keep)."""
            w = f32(k)
            n, kk = w.shape
            q = torch.empty(n, kk, dtype=torch.uint8, device=dev)
            sc = torch.empty(int(N.lib().vcap_mx_scale_bytes(n, kk)), dtype=torch.uint8, device=dev)
            N.check(N.lib().vcap_mx_quantize(N.DT_F32, w.data_ptr(), kk, n, kk, q.data_ptr(), sc.data_ptr(),
                                             _stream(dev)), "vcap_mx_quantize")
            return q, sc

        kstep = 32 if self.dt == N.DT_F32 else 64
        K = arch.patch_k
        self.kpad = ((K + 63) // 64) * 64 if kstep == 64 else ((K + 31) // 32) * 32
        pw = torch.zeros(arch.dim, self.kpad, dtype=torch.float32)
        pw[:, :K] = torch.from_numpy(np.ascontiguousarray(sd[p + "patch_embed.proj.weight"])).reshape(arch.dim, K)
        self._keep: List[torch.Tensor] = []
        keep = self._keep.append
        self.patch_w = pw.to(dev).to(tdt).contiguous()
        keep(self.patch_w)
        t = {
            "patch_b": f32(p + "patch_embed.proj.bias"),
            "cls": f32(p + "cls_token", (arch.dim,)),
            "pos": f32(p + "pos_embed", (arch.tokens, arch.dim)),
            "norm_g": f32(p + "norm.weight"), "norm_b": f32(p + "norm.bias"),
            "proj_w": f32("encoder.proj.weight"), "proj_b": f32("encoder.proj.bias"),
        }
        for v in t.values():
            keep(v)
        self.layers = (N.VitLayer * arch.depth)()
        for i in range(arch.depth):
            b = f"{p}blocks.{i}."
            lt = dict(ln1_g=f32(b + "norm1.weight"), ln1_b=f32(b + "norm1.bias"),
                      qkv_b=f32(b + "attn.qkv.bias"), proj_b=f32(b + "attn.proj.bias"),
                      ln2_g=f32(b + "norm2.weight"), ln2_b=f32(b + "norm2.bias"),
                      fc1_b=f32(b + "mlp.fc1.bias"), fc2_b=f32(b + "mlp.fc2.bias"))
            for name, key in (("qkv", "attn.qkv.weight"), ("proj", "attn.proj.weight"), ("fc1", "mlp.fc1.weight"),
                              ("fc2", "mlp.fc2.weight")):
                if name in self.mx_gemms:
                    lt[name + "_w"], lt[name + "_ws"] = wmx(b + key)
                else:
                    lt[name + "_w"] = wt(b + key)
            for k, v in lt.items():
                keep(v)
                setattr(self.layers[i], k, v.data_ptr())
        self.desc = N.VitDesc(dtype=self.dt, dim=arch.dim, depth=arch.depth, heads=arch.heads, patch=arch.patch,
                              image=arch.image, mlp=arch.mlp, video_dim=video_dim, kpad=self.kpad,
                              ln_eps=arch.ln_eps, patch_w=self.patch_w.data_ptr(), patch_b=t["patch_b"].data_ptr(),
                              cls=t["cls"].data_ptr(), pos=t["pos"].data_ptr(), norm_g=t["norm_g"].data_ptr(),
                              norm_b=t["norm_b"].data_ptr(), proj_w=t["proj_w"].data_ptr(),
                              proj_b=t["proj_b"].data_ptr(), layers=self.layers)
        self.ws = _Workspace(dev)

    def workspace_bytes(self, B: int, T: int) -> int:
        return int(N.lib().vcap_vit_workspace_bytes(C.byref(self.desc), B, T))

    def fuses_qkv_attention(self, layer: int = 0) -> bool:
        """Whether vcap_vit_encode runs this block's QKV projection + attention as one kernel (the
        library's own predicate, vcap_vit_layer_fuses_qkv_attention)."""
        rc = int(N.lib().vcap_vit_layer_fuses_qkv_attention(C.byref(self.desc), int(layer)))
        N.check(min(rc, 0), "vcap_vit_layer_fuses_qkv_attention")
        return rc == 1

    def encode(self, video: torch.Tensor, prefix: Optional["HipPrefix"] = None,
               out_prefix: Optional[torch.Tensor] = None):
        """video [B,T,3,H,W] (or [B,3,H,W]) f32 on device -> (enc_out [B,256] f32, prefix [B,P,E] f32|None)."""
        if video.dim() == 4:
            video = video.unsqueeze(1)
        if video.dim() != 5:
            raise ValueError(f"expect [B,T,3,H,W], got {tuple(video.shape)}")
        B, T, Cc, H, W = video.shape
        a = self.arch
        if Cc != 3 or H != a.image or W != a.image:
            raise ValueError(f"expect frames of 3x{a.image}x{a.image}, got {tuple(video.shape)}")
        if video.device != self.device and not (video.is_cuda and self.device.type == "cuda"):
            raise ValueError("video must be on the encoder's device")
        video = video.to(torch.float32).contiguous()
        enc = torch.empty(B, self.video_dim, dtype=torch.float32, device=video.device)
        pre = None
        pd = None
        if prefix is not None:
            shape = (B, prefix.prefix_len, prefix.n_embd)
            if out_prefix is not None:
                if tuple(out_prefix.shape) != shape or out_prefix.dtype != torch.float32 or not out_prefix.is_contiguous():
                    raise ValueError(f"out_prefix must be contiguous f32 {shape}")
                pre = out_prefix
            else:
                pre = torch.empty(*shape, dtype=torch.float32, device=video.device)
            pd = C.byref(prefix.desc)
        nbytes = self.workspace_bytes(B, T)
        ws = self.ws.get(nbytes)
        N.check(N.lib().vcap_vit_encode(C.byref(self.desc), pd, video.data_ptr(), B, T, enc.data_ptr(),
                                        N.ptr(pre), ws.data_ptr(), ws.numel(), _stream(video.device)),
                "vcap_vit_encode")
        return enc, pre


class HipPrefix:
    """Engine prefix normalisation (core/engine.py:44-50) + mapper (text_decoder.py:249)."""

    def __init__(self, sd: Dict[str, np.ndarray], n_embd: int, prefix_len: int = 4, ln_scale: float = 0.6,
                 in_weight: float = 0.4, device="cuda"):
        dev = torch.device(device)
        self.prefix_len, self.n_embd = prefix_len, n_embd
        self.mapper_w = torch.from_numpy(np.ascontiguousarray(sd["decoder.mapper.0.weight"], np.float32)).to(dev)
        self.mapper_b = torch.from_numpy(np.ascontiguousarray(sd["decoder.mapper.0.bias"], np.float32)).to(dev)
        if self.mapper_w.shape[0] != prefix_len * n_embd:
            raise ValueError(f"mapper out {self.mapper_w.shape[0]} != prefix_len*n_embd {prefix_len * n_embd}")
        self.set_scales(ln_scale, in_weight)

    def set_scales(self, ln_scale: Optional[float], in_weight: Optional[float]) -> None:
        self.ln_scale = float(ln_scale) if ln_scale is not None else 0.0
        self.in_weight = float(in_weight) if in_weight is not None else 0.0
        self.desc = N.PrefixDesc(ln_scale=self.ln_scale, in_weight=self.in_weight, prefix_len=self.prefix_len,
                                 n_embd=self.n_embd, mapper_w=self.mapper_w.data_ptr(),
                                 mapper_b=self.mapper_b.data_ptr())

    def project(self, emb: torch.Tensor) -> torch.Tensor:
        """emb [B,256] or [B,1,256] f32 -> prefix embeds [B, P, E] (vcap_prefix_project)."""
        B = emb.shape[0]
        e = emb.reshape(B, -1).to(torch.float32).contiguous()
        out = torch.empty(B, self.prefix_len, self.n_embd, dtype=torch.float32, device=e.device)
        N.check(N.lib().vcap_prefix_project(e.data_ptr(), B, e.shape[1], C.byref(self.desc), out.data_ptr(),
                                            _stream(e.device)), "vcap_prefix_project")
        return out


@dataclass
class GenConfig:
    max_new_tokens: int = 24
    min_new_tokens: int = 8
    no_repeat_ngram_size: int = 3
    repetition_penalty: float = 1.1
    eos_token_id: int = 50256
    pad_token_id: int = 50256
    use_graph: bool = True
    max_blocks: int = 0      # >0: narrower decode grids (decode sharing the GPU with an encode)
    num_beams: int = 1       # >1: device beam search (vcap_gpt2_beam_search, presets precise / detailed)
    length_penalty: float = 1.0
    # sampling (presets natural / safe_sample): HF's do_sample = (num_beams == 1 and temperature != 1),
    # text_decoder.py:137; top_k 50 is the generation-config default the reference inherits
    temperature: float = 1.0
    top_k: int = 50
    top_p: float = 1.0
    seed: int = 0

    @property
    def do_sample(self) -> bool:
        return self.num_beams == 1 and self.temperature != 1.0

    @classmethod
    def raw_greedy(cls, max_new_tokens: int = 24, eos: int = 50256, use_graph: bool = True) -> "GenConfig":
        """benchmark_baseline.run_decoder_steps semantics: argmax, no processors, no min length."""
        return cls(max_new_tokens, 0, 0, 1.0, eos, eos, use_graph)


class HipGPT2Decoder:
    """GPT2LMHeadModel greedy generate from inputs_embeds (text_decoder.py:131-144) on the HIP path."""

    # |bf16-screen score - exact f32 score| <= SCREEN_C * ||h||_2 * ||w_v||_2.  bf16 round-to-nearest
    # has unit roundoff u = 2^-8 PER OPERAND, so rounding h and w gives |h~w~ - hw| <= (2u + u^2) |h||w|
    # per element (7.83e-3 summed, Cauchy-Schwarz); the two f32 dot products (the screen's MFMA sum and
    # the rescoring's fma chain, n_embd <= 1024 terms) add 2 x 1024 x 2^-24 each, doubled for an
    # accumulator that truncates (2.44e-4): 8.07e-3, and 1.6 % over it.  The runtime multiplies the
    # bound by max(rep, 1/rep) when a repetition penalty is active (a penalised negative score is
    # scaled by rep, its error with it: csrc/runtime.hip issue_decode).  Round 5 shipped c = 0.0043,
    # which counted 2^-8 for BOTH roundings; tests/test_gpu_lm_screen.py builds a near-tie that the
    # old constant gets wrong and this one does not.
    SCREEN_C = 0.0082

    def __init__(self, sd: Dict[str, np.ndarray], arch: GPT2Arch, precision: str = "bf16", device="cuda",
                 prefix_len: int = 4, screen: bool = True):
        """precision "fp32" with `screen`: a greedy step without requested logits runs the lm_head
        in bf16 as a screen and rescores the tokens it cannot rule out in f32 (csrc/decode.hip,
        vcap_decode_finalize_kernel<float, true>): the same exact-f32 argmax for half the bytes."""
        N.lib()
        self.arch, self.precision, self.device = arch, precision, torch.device(device)
        self.dt, tdt = _dtype(precision)
        self.prefix_len = prefix_len
        dev = self.device
        p = "decoder.model.transformer."
        self._keep: List[torch.Tensor] = []

        def f32(k):
            t = torch.from_numpy(np.ascontiguousarray(sd[k], dtype=np.float32)).to(dev).contiguous()
            self._keep.append(t)
            return t

        def conv_t(k):  # Conv1D [in, out] -> [out, in] -> rows-packed (vcap_rows_pack)
            t = torch.from_numpy(np.ascontiguousarray(sd[k], dtype=np.float32)).t().contiguous()
            return self._pack(t.to(dev).to(tdt).contiguous())

        self.wte = torch.from_numpy(np.ascontiguousarray(sd[p + "wte.weight"], np.float32)).to(dev).to(tdt)
        self.wte = self.wte.contiguous()
        self._keep.append(self.wte)
        self.lm_head = self._pack(self.wte)   # tied lm_head, packed copy
        screen_w, screen_bound = None, 0.0
        if self.dt == N.DT_F32 and screen:
            screen_w = self._pack(self.wte.to(torch.bfloat16).contiguous(), N.DT_BF16)
            wmax = float(torch.linalg.vector_norm(self.wte.double(), dim=1).max())
            screen_bound = self.SCREEN_C * wmax * (1.0 + 1e-6)
        self.screen = screen_w is not None
        self.wpe = f32(p + "wpe.weight")
        lnf_g, lnf_b = f32(p + "ln_f.weight"), f32(p + "ln_f.bias")
        self.layers = (N.GPT2Layer * arch.n_layer)()
        for i in range(arch.n_layer):
            b = f"{p}h.{i}."
            ly = self.layers[i]
            ly.ln1_g, ly.ln1_b = f32(b + "ln_1.weight").data_ptr(), f32(b + "ln_1.bias").data_ptr()
            ly.attn_w, ly.attn_b = conv_t(b + "attn.c_attn.weight").data_ptr(), f32(b + "attn.c_attn.bias").data_ptr()
            ly.aproj_w = conv_t(b + "attn.c_proj.weight").data_ptr()
            ly.aproj_b = f32(b + "attn.c_proj.bias").data_ptr()
            ly.ln2_g, ly.ln2_b = f32(b + "ln_2.weight").data_ptr(), f32(b + "ln_2.bias").data_ptr()
            ly.fc_w, ly.fc_b = conv_t(b + "mlp.c_fc.weight").data_ptr(), f32(b + "mlp.c_fc.bias").data_ptr()
            ly.mproj_w = conv_t(b + "mlp.c_proj.weight").data_ptr()
            ly.mproj_b = f32(b + "mlp.c_proj.bias").data_ptr()
        self.desc = N.GPT2Desc(dtype=self.dt, n_embd=arch.n_embd, n_layer=arch.n_layer, n_head=arch.n_head,
                               vocab=arch.vocab, n_positions=arch.n_positions, prefix_len=prefix_len,
                               ln_eps=arch.ln_eps, wte=self.wte.data_ptr(), lm_head=self.lm_head.data_ptr(),
                               wpe=self.wpe.data_ptr(),
                               lnf_g=lnf_g.data_ptr(), lnf_b=lnf_b.data_ptr(), layers=self.layers,
                               lm_head_screen=screen_w.data_ptr() if screen_w is not None else None,
                               screen_bound=screen_bound)
        self.ws = _Workspace(dev)
        self._stable = {}             # (B, max_new) -> persistent prefix / ids buffers (graph reuse)
        torch.cuda.synchronize(dev)   # packing ran on the current stream; decodes may use others

    def _pack(self, w: torch.Tensor, dt: Optional[int] = None) -> torch.Tensor:
        """[N, K] device weight -> rows-packed copy (MFMA-fragment order, csrc/decode.hip)."""
        dt = self.dt if dt is None else dt
        rows, k = w.shape
        nbytes = int(N.lib().vcap_rows_packed_bytes(dt, rows, k))
        if nbytes == 0:
            raise ValueError(f"cannot pack a [{rows}, {k}] weight (K must be a multiple of 32 bf16 / 16 f32)")
        packed = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
        N.check(N.lib().vcap_rows_pack(dt, w.data_ptr(), w.stride(0), rows, k, packed.data_ptr(),
                                       _stream(w.device)), "vcap_rows_pack")
        self._keep.append(packed)
        return packed

    def workspace_bytes(self, B: int, prompt_len: int, max_new: int) -> int:
        return int(N.lib().vcap_gpt2_workspace_bytes(C.byref(self.desc), B, self.prefix_len + prompt_len, max_new))

    def generate_ids(self, prefix: torch.Tensor, prompt_ids: Sequence[int], cfg: GenConfig,
                     out: Optional[torch.Tensor] = None, logits_out: Optional[torch.Tensor] = None,
                     workspace: Optional["_Workspace"] = None, lengths_out: Optional[torch.Tensor] = None,
                     warped_out: Optional[torch.Tensor] = None, force_ids: Optional[torch.Tensor] = None
                     ) -> torch.Tensor:
        """prefix [B,P,E] f32 device, prompt ids (BOS-only prompt = [eos]) -> int32 [B, max_new] EOS-padded.

        `workspace` (KV pages + decode scratch) defaults to the decoder's own; concurrent decodes on
        different streams pass one each (the captured graph is keyed on it).  cfg.num_beams > 1 runs
        the device beam search instead of greedy; `lengths_out` (int32 [B]) then receives each best
        hypothesis' length (HF returns the first max(lengths) columns)."""
        if cfg.num_beams > 1:
            return self._beam_ids(prefix, prompt_ids, cfg, out, workspace, lengths_out)
        B, P, E = prefix.shape
        if P != self.prefix_len or E != self.arch.n_embd:
            raise ValueError(f"prefix shape {tuple(prefix.shape)} != [B,{self.prefix_len},{self.arch.n_embd}]")
        prefix = prefix.to(torch.float32).contiguous()
        ids = list(int(i) for i in prompt_ids)
        mx = int(cfg.max_new_tokens)
        fresh = (out is None and logits_out is None and workspace is None and warped_out is None and force_ids is None
                 and cfg.use_graph)
        if fresh:
            # A replayed graph bakes in the prefix / ids addresses: a caller that hands over new
            # tensors every call (the engine path) decodes through persistent per-shape buffers,
            # so one captured graph serves every call of that shape; the caller gets a copy.
            key = (B, mx)
            if key not in self._stable:
                self._stable[key] = (torch.empty(B, P, E, dtype=torch.float32, device=self.device),
                                     torch.empty(B, mx, dtype=torch.int32, device=self.device))
            sp, so = self._stable[key]
            sp.copy_(prefix)
            self.generate_ids(sp, ids, cfg, out=so)
            return so.clone()
        if out is None:
            out = torch.empty(B, mx, dtype=torch.int32, device=prefix.device)
        if logits_out is not None and tuple(logits_out.shape) != (mx, B, self.arch.vocab):
            raise ValueError("logits_out must be [max_new, B, vocab] f32")
        if (warped_out is not None or force_ids is not None) and not cfg.do_sample:
            raise ValueError("warped_out / force_ids belong to the sampling mode (temperature != 1)")
        gp = N.GenParams(max_new_tokens=mx, min_new_tokens=int(cfg.min_new_tokens),
                         no_repeat_ngram_size=int(cfg.no_repeat_ngram_size),
                         repetition_penalty=float(cfg.repetition_penalty), eos_token_id=int(cfg.eos_token_id),
                         pad_token_id=int(cfg.pad_token_id), use_graph=int(bool(cfg.use_graph)),
                         max_blocks=int(cfg.max_blocks))
        arr = (C.c_int * max(len(ids), 1))(*ids)
        ws = (workspace or self.ws).get(self.workspace_bytes(B, len(ids), mx))
        if cfg.do_sample:
            if warped_out is not None and (tuple(warped_out.shape) != (mx, B, self.arch.vocab)
                                           or warped_out.dtype != torch.float32 or not warped_out.is_contiguous()):
                raise ValueError("warped_out must be contiguous f32 [max_new, B, vocab]")
            if force_ids is not None:
                if tuple(force_ids.shape) != (B, mx):
                    raise ValueError("force_ids must be [B, max_new]")
                force_ids = force_ids.to(device=prefix.device, dtype=torch.int32).contiguous()
            sp = N.SampleParams(temperature=float(cfg.temperature), top_k=int(cfg.top_k), top_p=float(cfg.top_p),
                                seed=int(cfg.seed) & 0xFFFFFFFFFFFFFFFF)
            N.check(N.lib().vcap_gpt2_sample(C.byref(self.desc), C.byref(gp), C.byref(sp), prefix.data_ptr(), arr,
                                             len(ids), B, out.data_ptr(), N.ptr(logits_out), N.ptr(warped_out),
                                             N.ptr(force_ids), ws.data_ptr(), ws.numel(), _stream(prefix.device)),
                    "vcap_gpt2_sample")
            return out
        N.check(N.lib().vcap_gpt2_generate(C.byref(self.desc), C.byref(gp), prefix.data_ptr(), arr, len(ids), B,
                                           out.data_ptr(), N.ptr(logits_out), ws.data_ptr(), ws.numel(),
                                           _stream(prefix.device)), "vcap_gpt2_generate")
        return out


    def _beam_ids(self, prefix, prompt_ids, cfg: GenConfig, out, workspace, lengths_out):
        B, P, E = prefix.shape
        if P != self.prefix_len or E != self.arch.n_embd:
            raise ValueError(f"prefix shape {tuple(prefix.shape)} != [B,{self.prefix_len},{self.arch.n_embd}]")
        ids = [int(i) for i in prompt_ids]
        mx = int(cfg.max_new_tokens)
        prefix = prefix.to(torch.float32).contiguous()
        out = out if out is not None else torch.empty(B, mx, dtype=torch.int32, device=prefix.device)
        if lengths_out is None:
            lengths_out = torch.empty(B, dtype=torch.int32, device=prefix.device)
        S0 = self.prefix_len + len(ids)
        nbytes = int(N.lib().vcap_gpt2_beam_search_workspace_bytes(C.byref(self.desc), B, int(cfg.num_beams), S0, mx))
        if nbytes == 0:
            raise ValueError("vcap_gpt2_beam_search_workspace_bytes: unsupported shape")
        ws = (workspace or self.ws).get(nbytes)
        bp = N.BeamParams(num_beams=int(cfg.num_beams), max_new_tokens=mx, min_new_tokens=int(cfg.min_new_tokens),
                          no_repeat_ngram_size=int(cfg.no_repeat_ngram_size),
                          repetition_penalty=float(cfg.repetition_penalty), length_penalty=float(cfg.length_penalty),
                          early_stopping=0, eos_token_id=int(cfg.eos_token_id), use_graph=int(bool(cfg.use_graph)),
                          max_blocks=int(cfg.max_blocks))
        arr = (C.c_int * max(len(ids), 1))(*ids)
        N.check(N.lib().vcap_gpt2_beam_search(C.byref(self.desc), C.byref(bp), prefix.data_ptr(), arr, len(ids), B,
                                              out.data_ptr(), lengths_out.data_ptr(), ws.data_ptr(), ws.numel(),
                                              _stream(prefix.device)), "vcap_gpt2_beam_search")
        return out


def trim_generated(ids: torch.Tensor, eos: int) -> List[List[int]]:
    """HF generate output length: it stops after the first step where every row has finished
    (generation/utils.py stopping criteria); rows finished earlier are EOS-padded."""
    a = ids.cpu().numpy()
    B, L = a.shape
    fin = np.zeros(B, dtype=bool)
    stop = L
    for s in range(L):
        fin |= a[:, s] == eos
        if fin.all():
            stop = s + 1
            break
    return [list(map(int, a[b, :stop])) for b in range(B)]


def raw_greedy_tokens(ids: torch.Tensor, eos: int) -> List[List[int]]:
    """benchmark_baseline.run_decoder_steps bookkeeping: tokens up to and including the first EOS."""
    out = []
    for row in ids.cpu().numpy().tolist():
        toks = []
        for t in row:
            toks.append(int(t))
            if t == eos:
                break
        out.append(toks)
    return out
