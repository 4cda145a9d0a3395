"""InferenceEngine with the reference's surface (core/engine.py:20-83) on the HIP runtime.

_generate_once(video, prompt, **decode_kwargs) and infer(frames_dir) behave as the reference's:
encoder -> proj -> layer_norm(emb) * ln_scale * in_weight -> decoder.generate(preset kwargs) ->
clean_text; infer() runs the three configured candidates and select_best.  The encoder +
LN-scale + mapper run as one fused HIP call, and infer() encodes the video ONCE for its three
candidates (the reference re-runs the ViT per candidate, core/engine.py:43; results identical).
"""
from __future__ import annotations

import logging
from typing import List, Sequence

import torch

from core.config import InferenceConfig
from core.datatypes import CaptionCandidates, InferenceResult
from core.inference import preset_to_kwargs
from core.models.model_loader import load_caption_model
from core.postprocessing.candidate_ranker import select_best
from core.postprocessing.text_cleaner import clean_text
from core.preprocessing.frame_loader import load_video_tensor

log = logging.getLogger(__name__)


class InferenceEngine:
    def __init__(self, config: InferenceConfig):
        self.config = config
        self.device = config.device
        self.model = load_caption_model(config)

    @classmethod
    def from_config(cls, config: InferenceConfig):
        return cls(config)

    def _prefix(self, video: torch.Tensor) -> torch.Tensor:
        _, prefix = self.model.encode_prefix(video, self.config.ln_scale, self.config.in_weight)
        return prefix

    def _decode(self, prefix: torch.Tensor, prompt: str, **decode_kwargs) -> str:
        dec = self.model.decoder
        rows = dec.generate_from_prefix(
            prefix, dec.tokenizer.encode_prompt(prompt or ""),
            max_new_tokens=decode_kwargs.get("max_new_tokens", 24), num_beams=decode_kwargs.get("num_beams", 3),
            temperature=decode_kwargs.get("temperature", 1.0), top_p=decode_kwargs.get("top_p", 1.0),
            no_repeat_ngram_size=decode_kwargs.get("no_repeat_ngram_size", 3),
            repetition_penalty=decode_kwargs.get("repetition_penalty", 1.1), min_new_tokens=8,
            seed=self.config.sample_seed)
        text = dec.tokenizer.batch_decode(rows[:1], skip_special_tokens=True)
        return clean_text(text[0].strip() if text else "")

    @torch.no_grad()
    def _generate_once(self, video: torch.Tensor, prompt: str, **decode_kwargs) -> str:
        return self._decode(self._prefix(video), prompt, **decode_kwargs)

    @torch.no_grad()
    def infer(self, frames_dir: str) -> InferenceResult:
        video = load_video_tensor(frames_dir, num_frames=self.config.num_frames, image_size=self.config.image_size,
                                  device=self.device)
        return self.infer_video(video)

    @torch.no_grad()
    def infer_video(self, video: torch.Tensor) -> InferenceResult:
        prefix = self._prefix(video)
        c = self.config
        cands = CaptionCandidates(
            s1=self._decode(prefix, c.prompt1, **preset_to_kwargs(c.preset1)),
            s2=self._decode(prefix, c.prompt2, **preset_to_kwargs(c.preset2)),
            s3=self._decode(prefix, c.prompt3, **preset_to_kwargs(c.preset3)),
        )
        key, text, _ = select_best([("S1", cands.s1), ("S2", cands.s2), ("S3", cands.s3)])
        return InferenceResult(candidates=cands, best_key=key, best_text=text)

    def _decode_rows(self, prefix: torch.Tensor, prompt: str, **decode_kwargs) -> List[str]:
        """_decode for every row of a batched prefix: greedy rows and beam hypotheses evolve per
        sequence, so each row's caption equals its single-video decode (sampling draws from one
        generator for the whole batch: distributional parity only, as for single videos)."""
        dec = self.model.decoder
        rows = dec.generate_from_prefix(
            prefix, dec.tokenizer.encode_prompt(prompt or ""),
            max_new_tokens=decode_kwargs.get("max_new_tokens", 24), num_beams=decode_kwargs.get("num_beams", 3),
            temperature=decode_kwargs.get("temperature", 1.0), top_p=decode_kwargs.get("top_p", 1.0),
            no_repeat_ngram_size=decode_kwargs.get("no_repeat_ngram_size", 3),
            repetition_penalty=decode_kwargs.get("repetition_penalty", 1.1), min_new_tokens=8,
            seed=self.config.sample_seed)
        return [clean_text(t.strip()) for t in dec.tokenizer.batch_decode(rows, skip_special_tokens=True)]

    @torch.no_grad()
    def infer_videos(self, videos: torch.Tensor) -> List[InferenceResult]:
        """infer_video over a batch [B, T, 3, H, W]: ONE fused encode for all B videos and one
        batched decode per candidate (the serving path coalesces requests into this call)."""
        prefix = self._prefix(videos)
        c = self.config
        s1 = self._decode_rows(prefix, c.prompt1, **preset_to_kwargs(c.preset1))
        s2 = self._decode_rows(prefix, c.prompt2, **preset_to_kwargs(c.preset2))
        s3 = self._decode_rows(prefix, c.prompt3, **preset_to_kwargs(c.preset3))
        out = []
        for a, b, d in zip(s1, s2, s3):
            key, text, _ = select_best([("S1", a), ("S2", b), ("S3", d)])
            out.append(InferenceResult(candidates=CaptionCandidates(s1=a, s2=b, s3=d), best_key=key, best_text=text))
        return out

    def load_video(self, frames_dir: str) -> torch.Tensor:
        """frames_dir -> [1, T, 3, H, W] on the engine's device (core/preprocessing/frame_loader.py)."""
        return load_video_tensor(frames_dir, num_frames=self.config.num_frames, image_size=self.config.image_size,
                                 device=self.device)

    def max_batch_videos(self) -> int:
        """Videos one device call decodes at once: a greedy / sampling candidate's prefill takes
        B * (prefix_len + prompt_len) decoder rows, within vcap_gpt2_max_rows(); a beam candidate
        is chunked by the decoder itself (vcap.search.beam_search_any), so this only sizes the
        coalesced batch to what one device beam chunk takes - at most 8 sequences and
        B * num_beams * (prefix_len + prompt_len) rows - to keep every chunk full."""
        from vcap import _native as N
        from vcap.search import BEAM_DEVICE_MAX_B
        c, tok = self.config, self.model.decoder.tokenizer
        rows = limit = int(N.lib().vcap_gpt2_max_rows())
        for prompt, preset in ((c.prompt1, c.preset1), (c.prompt2, c.preset2), (c.prompt3, c.preset3)):
            try:
                s0 = c.prefix_len + len(tok.encode_prompt(prompt or ""))
            except ValueError:
                s0 = c.prefix_len + 1   # an untokenizable prompt fails per request anyway
            beams = max(1, preset_to_kwargs(preset).get("num_beams", 1))
            rows = min(rows, limit // s0)
            if beams > 1:
                rows = min(rows, BEAM_DEVICE_MAX_B, limit // (beams * s0))
        return max(1, rows)

    @torch.no_grad()
    def infer_batch(self, frames_dirs: Sequence[str]) -> List[InferenceResult]:
        """infer() for several frames directories in one engine call (each video's frames share a
        size; videos are preprocessed on the GPU one by one and encoded/decoded together)."""
        vids = [load_video_tensor(d, num_frames=self.config.num_frames, image_size=self.config.image_size,
                                  device=self.device) for d in frames_dirs]
        return self.infer_videos(torch.cat(vids, dim=0))
