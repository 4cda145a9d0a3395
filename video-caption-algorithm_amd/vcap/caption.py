"""`VideoCaptionModel`-shaped object on the HIP runtime (the drop-in boundary of SURVEY.md §8b).

Surface kept from the reference (src/models/caption_model.py:11-101, text_decoder.py:12-146):
  model.encoder(video)            -> [B, 256] f32       (ViTFrameEncoder.forward)
  model.proj(emb)                 -> emb                (Identity, proj_hidden=0)
  model.decoder.mapper(emb)       -> [B, P*E] f32       (Linear 256 -> P*E; Dropout is eval-identity)
  model.decoder.generate(emb, prompt, **kw) -> list[str]   (HF generate semantics, see below)
  model.decoder.tokenizer / .cond_mode / .prefix_len / .model.config.n_embd / .model.transformer.wte
  model.decoder.model(inputs_embeds=, attention_mask=, past_key_values=, use_cache=True)
                                  (GPT2LMHeadModel forward as benchmark_baseline.py:160-240 calls it)
  model.generate(video, prompt, **kw)       (VideoCaptionModel.generate: no engine LN-scale)
plus the batched fast path `generate_ids(video, prompt_ids, ...)` -> int32 [B, max_new] on device.

Decode semantics of decoder.generate (text_decoder.py:131-144): num_beams == 1 and temperature == 1
-> greedy with RepetitionPenalty, NoRepeatNGram and min_new_tokens (on device, one hipGraph);
num_beams > 1 -> beam search; num_beams == 1 and temperature != 1 -> sampling (temperature, top-k 50,
top-p; on device, one hipGraph).
"""
from __future__ import annotations

import ctypes as C
import logging
from types import SimpleNamespace
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native as N
from . import configs
from .model import GenConfig, HipGPT2Decoder, HipPrefix, HipViTEncoder, trim_generated
from .tokenizer import load_tokenizer
from .weights import normalize_checkpoint, synthetic_state_dict

log = logging.getLogger(__name__)


class _Encoder:
    def __init__(self, hip: HipViTEncoder):
        self.hip = hip

    def __call__(self, video: torch.Tensor) -> torch.Tensor:
        emb, _ = self.hip.encode(video, None)
        return emb


class _Identity:
    def __call__(self, x):
        return x


class _WTE:
    """decoder.model.transformer.wte: the token embedding as the reference's nn.Embedding returns it
    (fp32 rows, core/scripts/benchmark_baseline.py:162-227 feeds them back as inputs_embeds).  The
    decoder's own table may be bf16 (the throughput mode); the fp32 rows are uploaded on first use."""

    def __init__(self, table: torch.Tensor, table_f32=None):
        self.weight = table
        self._src = table_f32       # host fp32 [V, E] (state dict) or None: use `table` as is
        self._f32 = None

    def __call__(self, ids: torch.Tensor) -> torch.Tensor:
        if self._src is not None and self._f32 is None:
            self._f32 = torch.from_numpy(np.ascontiguousarray(self._src, dtype=np.float32)).to(self.weight.device)
        t = self._f32 if self._f32 is not None else self.weight
        return t[ids.to(t.device)].float()


class HipPast:
    """`past_key_values` of the HIP decoder: the paged KV state lives in a workspace carved for
    `rows` sequences of S0 prefill positions + up to `capacity` appended ones."""

    def __init__(self, hip: HipGPT2Decoder, rows: int, S0: int, capacity: int):
        self.hip, self.rows, self.S0, self.capacity = hip, rows, S0, capacity
        nbytes = int(N.lib().vcap_gpt2_beam_workspace_bytes(C.byref(hip.desc), rows, S0, capacity))
        self.ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=hip.device)
        self.length = 0

    def get_seq_length(self) -> int:
        return self.length


class HipGPT2LMHead:
    """`decoder.model`: GPT2LMHeadModel's forward as core/scripts/benchmark_baseline.py:160-240
    drives it - `model(inputs_embeds=, attention_mask=, past_key_values=, use_cache=True,
    return_dict=True)` -> `.logits`, `.past_key_values` - on vcap_gpt2_forward_embeds.

    The first call (past_key_values None) prefills the whole `inputs_embeds` [B, L, E]; later
    calls append one position per row.  `.logits` holds the LAST position only ([B, 1, vocab]),
    which is what every caller reads (`outputs.logits[:, -1, :]`).  attention_mask must be all
    ones (no padding on this path)."""

    def __init__(self, hip: HipGPT2Decoder, arch: configs.GPT2Arch, wte: "_WTE", max_cache_tokens: int = 128):
        self.hip, self.arch = hip, arch
        self.config = SimpleNamespace(n_embd=arch.n_embd, n_layer=arch.n_layer, n_head=arch.n_head,
                                      vocab_size=arch.vocab)
        self.transformer = SimpleNamespace(wte=wte)
        self.max_cache_tokens = max_cache_tokens

    def __call__(self, input_ids=None, inputs_embeds=None, attention_mask=None, past_key_values=None,
                 use_cache: bool = True, return_dict: bool = True):
        if inputs_embeds is None:
            if input_ids is None:
                raise ValueError("give input_ids or inputs_embeds")
            inputs_embeds = self.transformer.wte(input_ids)
        x = inputs_embeds.to(self.hip.device, torch.float32).contiguous()
        B, L, E = x.shape
        if E != self.arch.n_embd:
            raise ValueError(f"inputs_embeds last dim {E} != n_embd {self.arch.n_embd}")
        if attention_mask is not None and not bool((attention_mask != 0).all()):
            raise NotImplementedError("padded attention masks are not supported on the HIP decode path")
        past = past_key_values
        if past is None:
            cap = min(self.max_cache_tokens, self.arch.n_positions - L)
            past = HipPast(self.hip, B, L, cap)
        elif not isinstance(past, HipPast):
            raise TypeError("past_key_values must come from a previous call of this model")
        elif L != 1 or B != past.rows:
            raise ValueError("after the prefill, feed one position per row ([rows, 1, E])")
        elif past.length >= past.S0 + past.capacity:
            raise ValueError(f"KV capacity exhausted ({past.capacity} appended positions; raise max_cache_tokens)")
        logits = torch.empty(B, self.arch.vocab, dtype=torch.float32, device=self.hip.device)
        N.check(N.lib().vcap_gpt2_forward_embeds(C.byref(self.hip.desc), x.data_ptr(), B, L, past.length, past.S0,
                                                 past.capacity, logits.data_ptr(), past.ws.data_ptr(),
                                                 past.ws.numel(), torch.cuda.current_stream(self.hip.device).cuda_stream),
                "vcap_gpt2_forward_embeds")
        past.length += L
        out = SimpleNamespace(logits=logits[:, None, :], past_key_values=past if use_cache else None)
        return out if return_dict else (out.logits, out.past_key_values)


class HipTextDecoder:
    def __init__(self, sd, arch: configs.GPT2Arch, precision: str, device, prefix_len: int = 4,
                 tokenizer_dir: str = "", use_graph: bool = True):
        self.arch, self.prefix_len, self.cond_mode = arch, prefix_len, "prefix"
        self.hip = HipGPT2Decoder(sd, arch, precision, device, prefix_len)
        self.mapper_op = HipPrefix(sd, arch.n_embd, prefix_len, 0.0, 0.0, device)
        self.tokenizer = load_tokenizer(tokenizer_dir, arch.eos_token_id)
        self.use_graph = use_graph
        self.model = HipGPT2LMHead(self.hip, arch, _WTE(self.hip.wte, sd["decoder.model.transformer.wte.weight"]))

    def mapper(self, emb: torch.Tensor) -> torch.Tensor:
        """Linear 256 -> P*E on the HIP path (cupy_linear_mapper / CuPyLinearCompat replacement)."""
        B = emb.shape[0]
        return self.mapper_op.project(emb).reshape(B, *emb.shape[1:-1], self.prefix_len * self.arch.n_embd)

    def prefix_embeds(self, emb: torch.Tensor) -> torch.Tensor:
        return self.mapper_op.project(emb)

    def generate_from_prefix(self, prefix: torch.Tensor, prompt_ids: Sequence[int], *, max_new_tokens: int = 32,
                             num_beams: int = 1, temperature: float = 1.0, top_p: float = 0.9,
                             no_repeat_ngram_size: int = 3, repetition_penalty: float = 1.15,
                             min_new_tokens: int = 8, seed: int = 0) -> List[List[int]]:
        eos = self.tokenizer.eos_token_id
        if num_beams == 1 and temperature == 1.0:
            cfg = GenConfig(max_new_tokens, min_new_tokens, no_repeat_ngram_size, repetition_penalty, eos, eos,
                            self.use_graph)
            ids = self.hip.generate_ids(prefix, prompt_ids, cfg)
            return trim_generated(ids, eos)
        from . import search
        if num_beams > 1:
            return search.beam_search_any(self.hip, prefix, prompt_ids, num_beams=num_beams,
                                             max_new_tokens=max_new_tokens, min_new_tokens=min_new_tokens,
                                             no_repeat_ngram_size=no_repeat_ngram_size,
                                             repetition_penalty=repetition_penalty, eos=eos,
                                             use_graph=self.use_graph)
        return search.sample(self.hip, prefix, prompt_ids, temperature=temperature, top_p=top_p,
                             max_new_tokens=max_new_tokens, min_new_tokens=min_new_tokens,
                             no_repeat_ngram_size=no_repeat_ngram_size, repetition_penalty=repetition_penalty,
                             eos=eos, seed=seed, use_graph=self.use_graph)

    @torch.no_grad()
    def generate(self, video_emb: torch.Tensor, prompt: str = "", max_new_tokens: int = 32, num_beams: int = 1,
                 temperature: float = 1.0, top_p: float = 0.9, no_repeat_ngram_size: int = 3,
                 repetition_penalty: float = 1.15, min_new_tokens: int = 8) -> List[str]:
        """GPT2TextDecoder.generate (text_decoder.py:105-146): video_emb [B,256] or [B,1,256]."""
        prompt_ids = self.tokenizer.encode_prompt(prompt)
        prefix = self.prefix_embeds(video_emb)
        rows = self.generate_from_prefix(prefix, prompt_ids, max_new_tokens=max_new_tokens, num_beams=num_beams,
                                         temperature=temperature, top_p=top_p,
                                         no_repeat_ngram_size=no_repeat_ngram_size,
                                         repetition_penalty=repetition_penalty, min_new_tokens=min_new_tokens)
        return [t.strip() for t in self.tokenizer.batch_decode(rows, skip_special_tokens=True)]


def resolve_decoder_precision(precision: str, decoder_precision: str = "auto") -> str:
    """The GPT-2 decoder's arithmetic.  "auto" = fp32 whatever the ViT runs in: the reference's own
    split - its ViT under half-precision autocast (src/models/video_encoder.py:261-264,
    backend_config.py:46), its decoder always fp32 (src/models/text_decoder.py:131-144) - so the
    drop-in surface decodes token-exactly by default.  "bf16" is the throughput mode (BASELINE
    configs[1] line of bench.py)."""
    if decoder_precision == "auto":
        return "fp32"
    if decoder_precision not in ("bf16", "fp32"):
        raise ValueError(f"decoder_precision must be auto, bf16 or fp32, got {decoder_precision!r}")
    return decoder_precision


class HipVideoCaptionModel:
    def __init__(self, sd, vit_name: str = "vit_base_patch16_224", gpt2_name: str = "gpt2", prefix_len: int = 4,
                 precision: str = "bf16", device="cuda", tokenizer_dir: str = "", use_graph: bool = True,
                 decoder_precision: str = "auto"):
        """precision: the ViT's operand type (bf16 / fp32 / fp8 = MXFP8 block GEMMs); decoder_precision:
        see resolve_decoder_precision (default fp32, the reference's decoder arithmetic)."""
        self.device = torch.device(device)
        self.vit_arch, self.gpt2_arch = configs.vit_arch(vit_name), configs.gpt2_arch(gpt2_name)
        self.hip_encoder = HipViTEncoder(sd, self.vit_arch, precision, self.device)
        self.encoder = _Encoder(self.hip_encoder)
        self.proj = _Identity()
        self.decoder_precision = resolve_decoder_precision(precision, decoder_precision)
        self.decoder = HipTextDecoder(sd, self.gpt2_arch, self.decoder_precision, self.device, prefix_len,
                                      tokenizer_dir, use_graph)
        self._engine_prefix = HipPrefix(sd, self.gpt2_arch.n_embd, prefix_len, 0.6, 0.4, self.device)

    def encode_prefix(self, video: torch.Tensor, ln_scale: Optional[float], in_weight: Optional[float]):
        """Fused encoder -> proj -> engine LN-scale -> mapper (core/engine.py:43-50 + text_decoder.py:249)."""
        self._engine_prefix.set_scales(ln_scale if ln_scale and ln_scale > 0 else 0.0,
                                       in_weight if in_weight and in_weight > 0 else 0.0)
        return self.hip_encoder.encode(video.to(self.device), self._engine_prefix)

    @torch.no_grad()
    def generate(self, video: torch.Tensor, prompt: str = "", **gen_kwargs) -> List[str]:
        """VideoCaptionModel.generate (caption_model.py:93-101): encoder -> proj -> decoder.generate."""
        emb = self.proj(self.encoder(video.to(self.device)))
        return self.decoder.generate(emb, prompt=prompt, **gen_kwargs)

    @torch.no_grad()
    def generate_ids(self, video: torch.Tensor, prompt_ids: Sequence[int], *, ln_scale: float = 0.6,
                     in_weight: float = 0.4, cfg: Optional[GenConfig] = None) -> torch.Tensor:
        """Batched fast path: int32 [B, max_new] EOS-padded greedy ids on device."""
        _, prefix = self.encode_prefix(video, ln_scale, in_weight)
        eos = self.gpt2_arch.eos_token_id
        cfg = cfg or GenConfig(24, 8, 3, 1.1, eos, eos, self.decoder.use_graph)
        return self.decoder.hip.generate_ids(prefix, list(prompt_ids), cfg)


def build_state_dict(ckpt: str, vit_name: str, gpt2_name: str, weights_seed: Optional[int], prefix_len: int = 4):
    """Reference checkpoint or seeded random init (core/models/model_loader.py:31-80).

    Same acceptance as the reference: a raw state_dict or {"model_state": ...}, loaded with
    strict=False - keys the checkpoint lacks keep the model's initial values (here the seeded
    initialiser's; the reference's come from the pretrained timm / HF weights it fetches) and are
    logged (at most 6 names), unexpected keys are logged and ignored, a shape mismatch raises as
    load_state_dict does.  Deviation: no `weights_only=False` retry - a checkpoint that the safe
    loader refuses is rejected rather than unpickled."""
    seed = 1 if weights_seed is None else int(weights_seed)
    init = synthetic_state_dict(seed, configs.vit_arch(vit_name), configs.gpt2_arch(gpt2_name), prefix_len)
    if not ckpt:
        return init
    try:
        state = torch.load(ckpt, map_location="cpu", weights_only=True)
    except Exception as e:   # noqa: BLE001  (the reference logs and retries unsafely; we refuse)
        raise RuntimeError(f"cannot load {ckpt} with torch.load(weights_only=True): {e}") from e
    sd = normalize_checkpoint(state)
    missing = [k for k in init if k not in sd]
    unexpected = [k for k in sd if k not in init]
    for k in init:
        if k in sd and tuple(sd[k].shape) != tuple(init[k].shape):
            raise ValueError(f"size mismatch for {k}: checkpoint {tuple(sd[k].shape)} vs model {tuple(init[k].shape)}")
    if missing:
        log.warning("missing keys (kept at init): %d, e.g. %s", len(missing), missing[:6])
    if unexpected:
        log.warning("unexpected keys (ignored): %d, e.g. %s", len(unexpected), unexpected[:6])
    return {k: sd.get(k, v) for k, v in init.items()}


def synthetic_keys(vit_name: str, gpt2_name: str, prefix_len: int = 4) -> List[str]:
    va, ga = configs.vit_arch(vit_name), configs.gpt2_arch(gpt2_name)
    keys = ["encoder.backbone.cls_token", "encoder.backbone.pos_embed", "encoder.backbone.patch_embed.proj.weight",
            "encoder.proj.weight", "decoder.model.transformer.wte.weight", "decoder.mapper.0.weight"]
    keys += [f"encoder.backbone.blocks.{i}.attn.qkv.weight" for i in range(va.depth)]
    keys += [f"decoder.model.transformer.h.{i}.attn.c_attn.weight" for i in range(ga.n_layer)]
    return keys
