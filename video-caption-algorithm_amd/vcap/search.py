"""Beam search and sampling over the HIP step-wise decode ABI (vcap_gpt2_prefill / _step / _reorder).

The forward passes (prefill, one token per row per step, KV-cache row permutation) run in
libvcap_hip.so; this module keeps the search bookkeeping as small device tensor ops.

`beam_search_device` runs the whole search in libvcap_hip.so (csrc/beam.hip, one hipGraph); the
host-bookkeeping `beam_search` below is its cross-check (tests/test_gpu_search.py).

Beam search restates transformers 5.15.0 `GenerationMixin._beam_search` (the only copy in this
image; the reference pins 4.57.1) as the reference reaches it from
text_decoder.py:131-144 with inputs_embeds (decoder_prompt_len = 0): log_softmax -> processors
(RepetitionPenalty, NoRepeatNGram, MinLength/MinNewTokens) -> + running scores -> top-2k over
beams x vocab -> running / finished beam updates with length_penalty=1.0, early_stopping=False
-> cache reorder.  Sampling restates `_sample` with TemperatureLogitsWarper + TopKLogitsWarper(50) + TopPLogitsWarper;
it runs on the device (csrc/sample.hip); its RNG stream is Philox, so parity with the reference is
distributional only; `sampling_scores` is the torch restatement of the warped scores (test reference).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence

import torch
import torch.nn.functional as F

from . import _native as N


class _StepState:
    def __init__(self, dec, rows: int, S0: int, max_new: int):
        self.dec, self.rows, self.S0, self.max_new = dec, rows, S0, max_new
        nbytes = int(N.lib().vcap_gpt2_beam_workspace_bytes(C.byref(dec.desc), rows, S0, max_new))
        self.ws = dec.ws.get(nbytes)
        self.stream = torch.cuda.current_stream(dec.device).cuda_stream

    def prefill(self, prefix: torch.Tensor, prompt_ids: Sequence[int]) -> torch.Tensor:
        B = prefix.shape[0]
        logits = torch.empty(B, self.dec.arch.vocab, dtype=torch.float32, device=prefix.device)
        arr = (C.c_int * max(len(prompt_ids), 1))(*prompt_ids)
        N.check(N.lib().vcap_gpt2_prefill(C.byref(self.dec.desc), prefix.contiguous().data_ptr(), arr, len(prompt_ids),
                                          B, self.rows, self.max_new, logits.data_ptr(), self.ws.data_ptr(),
                                          self.ws.numel(), self.stream), "vcap_gpt2_prefill")
        return logits

    def step(self, tokens: torch.Tensor, pos: int) -> torch.Tensor:
        tok = tokens.to(torch.int32).contiguous()
        logits = torch.empty(self.rows, self.dec.arch.vocab, dtype=torch.float32, device=tok.device)
        N.check(N.lib().vcap_gpt2_step(C.byref(self.dec.desc), tok.data_ptr(), self.rows, self.S0, self.max_new, pos,
                                       logits.data_ptr(), self.ws.data_ptr(), self.ws.numel(), self.stream),
                "vcap_gpt2_step")
        return logits

    def reorder(self, src_rows: torch.Tensor, length: int) -> None:
        src = src_rows.to(torch.int32).contiguous()
        N.check(N.lib().vcap_gpt2_reorder(C.byref(self.dec.desc), src.data_ptr(), self.rows, self.S0, self.max_new,
                                          length, self.ws.data_ptr(), self.ws.numel(), self.stream),
                "vcap_gpt2_reorder")


@torch.no_grad()
def beam_search_device(dec, prefix: torch.Tensor, prompt_ids: Sequence[int], *, num_beams: int, max_new_tokens: int,
                       min_new_tokens: int = 8, no_repeat_ngram_size: int = 3, repetition_penalty: float = 1.1,
                       eos: int = 50256, length_penalty: float = 1.0, use_graph: bool = True,
                       max_blocks: int = 0) -> List[List[int]]:
    """The same search as `beam_search`, entirely on the device (vcap_gpt2_beam_search through
    HipGPT2Decoder.generate_ids: fused log_softmax / processor / top-2k kernels and a device
    bookkeeping kernel, one hipGraph, one device->host copy of the result).  Persistent
    per-shape prefix / output buffers keep the captured graph across calls.  max_blocks > 0 caps
    the step's GEMV grids and the beam lm_head's grid (a search sharing the GPU with an encode)."""
    from .model import GenConfig
    B, P, E = prefix.shape
    cache = dec.__dict__.setdefault("_beam_bufs", {})   # persistent per decoder and shape
    key = (B, num_beams, max_new_tokens)
    if key not in cache:
        cache[key] = (torch.empty(B, P, E, dtype=torch.float32, device=prefix.device),
                      torch.empty(B, max_new_tokens, dtype=torch.int32, device=prefix.device),
                      torch.empty(B, dtype=torch.int32, device=prefix.device))
    pre, out, lens = cache[key]
    pre.copy_(prefix)
    cfg = GenConfig(max_new_tokens, min_new_tokens, no_repeat_ngram_size, repetition_penalty, eos, eos, use_graph,
                    num_beams=num_beams, length_penalty=length_penalty, max_blocks=max_blocks)
    dec.generate_ids(pre, prompt_ids, cfg, out=out, lengths_out=lens)
    ids = out.cpu()
    n = int(lens.max().item())
    return [list(map(int, r)) for r in ids[:, :n].tolist()]


BEAM_DEVICE_MAX_B = 8   # sequences per device beam-search call (csrc/beam.hip select kernel: one wave each)


@torch.no_grad()
def beam_search_any(dec, prefix: torch.Tensor, prompt_ids: Sequence[int], *, num_beams: int, max_new_tokens: int,
                    min_new_tokens: int = 8, no_repeat_ngram_size: int = 3, repetition_penalty: float = 1.1,
                    eos: int = 50256, length_penalty: float = 1.0, use_graph: bool = True) -> List[List[int]]:
    """Beam search for any batch: sequences go to the device search (one hipGraph) in chunks within
    its limits (<= 8 sequences, B * num_beams * (prefix + prompt) <= vcap_gpt2_max_rows()); a shape
    the device search refuses (num_beams > 8 or too many candidates for the vocabulary, context
    > 128) runs the host-bookkeeping search over the same step kernels.  Sequences are independent
    in HF's search, so chunking changes nothing but the padding: rows are EOS-padded to the longest
    hypothesis of the whole batch, as one generate() call returns them."""
    B = prefix.shape[0]
    S0 = dec.prefix_len + len(prompt_ids)
    limit = int(N.lib().vcap_gpt2_max_rows())
    step = max(1, min(BEAM_DEVICE_MAX_B, limit // max(1, num_beams * S0)))
    kw = dict(num_beams=num_beams, max_new_tokens=max_new_tokens, min_new_tokens=min_new_tokens,
              no_repeat_ngram_size=no_repeat_ngram_size, repetition_penalty=repetition_penalty, eos=eos,
              length_penalty=length_penalty)
    rows: List[List[int]] = []
    device_ok = True
    for i in range(0, B, step):
        chunk = prefix[i:i + step]
        if device_ok:
            try:
                rows += beam_search_device(dec, chunk, prompt_ids, use_graph=use_graph, **kw)
                continue
            except N.VcapError as e:
                if e.rc != N.E_UNSUPPORTED:
                    raise
                device_ok = False
        host_step = max(1, min(chunk.shape[0], limit // max(1, num_beams), limit // max(1, S0)))
        for j in range(0, chunk.shape[0], host_step):
            rows += beam_search(dec, chunk[j:j + host_step], prompt_ids, **kw)
    width = max(len(r) for r in rows)
    return [r + [eos] * (width - len(r)) for r in rows]


def _processors(scores: torch.Tensor, seqs: torch.Tensor, rep: float, ngram: int, min_new: int, eos: int):
    """RepetitionPenalty -> NoRepeatNGram -> MinLength/MinNewTokens (prompt length 0) on [rows, V]."""
    L = seqs.shape[1]
    if rep != 1.0 and L > 0:
        g = torch.gather(scores, 1, seqs)
        scores = scores.scatter(1, seqs, torch.where(g < 0, g * rep, g / rep))
    if ngram and ngram > 0 and L >= ngram:
        # windows [rows, L-n+1, n]; a window bans its last token when its (n-1)-prefix equals the tail
        win = seqs.unfold(1, ngram, 1)
        tail = seqs[:, L - ngram + 1:] if ngram > 1 else seqs[:, :0]
        match = (win[:, :, :ngram - 1] == tail[:, None, :]).all(-1)
        if bool(match.any()):
            r, w = match.nonzero(as_tuple=True)
            scores = scores.index_put((r, win[r, w, ngram - 1]),
                                      torch.tensor(-float("inf"), dtype=scores.dtype, device=scores.device))
    if L < min_new:
        scores = scores.clone()
        scores[:, eos] = -float("inf")
    return scores


def _gather_beams(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    while idx.dim() < t.dim():
        idx = idx.unsqueeze(-1)
    return torch.take_along_dim(t, idx, dim=1)


@torch.no_grad()
def beam_search(dec, prefix: torch.Tensor, prompt_ids: Sequence[int], *, num_beams: int, max_new_tokens: int,
                min_new_tokens: int = 8, no_repeat_ngram_size: int = 3, repetition_penalty: float = 1.1,
                eos: int = 50256, length_penalty: float = 1.0, early_stopping=False) -> List[List[int]]:
    B, dev = prefix.shape[0], prefix.device
    nb, V = num_beams, dec.arch.vocab
    rows = B * nb
    S0 = dec.prefix_len + len(prompt_ids)
    st = _StepState(dec, rows, S0, max_new_tokens)
    logits0 = st.prefill(prefix, list(prompt_ids))
    st.reorder(torch.arange(rows, device=dev) // nb, S0)          # expand each sequence to its beams
    logits = logits0.repeat_interleave(nb, dim=0)

    max_length = max_new_tokens
    keep = 2 * nb
    top_mask = torch.cat([torch.ones(nb, dtype=torch.bool), torch.zeros(keep - nb, dtype=torch.bool)]).to(dev)
    running_seq = torch.full((B, nb, max_length), eos, dtype=torch.long, device=dev)
    sequences = running_seq.clone()
    running_scores = torch.zeros(B, nb, device=dev)
    running_scores[:, 1:] = -1e9
    beam_scores = torch.full((B, nb), -1e9, device=dev)
    finished = torch.zeros(B, nb, dtype=torch.bool, device=dev)
    unsat = torch.ones(B, 1, dtype=torch.bool, device=dev)
    running_bidx = torch.full((B, nb, max_length), -1, dtype=torch.int32, device=dev)
    beam_idx = running_bidx.clone()
    offsets = torch.arange(B, device=dev).view(-1, 1) * nb
    cur = 0
    while True:
        lp = F.log_softmax(logits.float(), dim=-1)
        lp = _processors(lp, running_seq[:, :, :cur].reshape(rows, cur), repetition_penalty, no_repeat_ngram_size,
                         min_new_tokens, eos)
        lp = (lp.view(B, nb, V) + running_scores[:, :, None]).reshape(B, nb * V)
        topk_lp, topk_i = torch.topk(lp, k=keep)
        src_beam = topk_i // V
        topk_bidx = _gather_beams(running_bidx, src_beam)
        topk_seq = _gather_beams(running_seq, src_beam)
        topk_ids = topk_i % V
        topk_seq[:, :, cur] = topk_ids
        topk_bidx[:, :, cur] = (src_beam + offsets).to(torch.int32)
        hits = (topk_ids == eos) | (cur + 1 >= max_length)
        # running beams for the next iteration
        run_lp = topk_lp + hits.float() * -1.0e9
        nxt = torch.topk(run_lp, k=nb)[1]
        running_seq = _gather_beams(topk_seq, nxt)
        running_scores = _gather_beams(run_lp, nxt)
        running_bidx = _gather_beams(topk_bidx, nxt)
        # finished hypotheses
        did = hits & top_mask[None, :]
        sc = topk_lp / ((cur + 1) ** length_penalty)
        full = torch.all(finished, dim=-1, keepdim=True) & (early_stopping is True)
        sc = sc + full.float() * -1.0e9 + (~unsat).float() * -1.0e9 + (~did).float() * -1.0e9
        m_seq = torch.cat([sequences, topk_seq], dim=1)
        m_sc = torch.cat([beam_scores, sc], dim=1)
        m_bidx = torch.cat([beam_idx, topk_bidx], dim=1)
        m_fin = torch.cat([finished, did], dim=1)
        sel = torch.topk(m_sc, k=nb)[1]
        sequences, beam_scores = _gather_beams(m_seq, sel), _gather_beams(m_sc, sel)
        beam_idx, finished = _gather_beams(m_bidx, sel), _gather_beams(m_fin, sel)
        # cache follows the surviving running beams
        st.reorder(running_bidx[:, :, cur].reshape(-1), S0 + cur)
        cur += 1
        if early_stopping == "never" and length_penalty > 0.0:
            best_len = max_length
        else:
            best_len = cur
        best_running = running_scores[:, :1] / (best_len ** length_penalty)
        worst_fin = torch.where(finished, torch.min(beam_scores, dim=1, keepdim=True)[0], torch.full_like(beam_scores, -1.0e9))
        unsat = unsat & torch.any(best_running > worst_fin, dim=-1, keepdim=True)
        go = bool(torch.any(unsat)) and not (bool(torch.all(finished)) and early_stopping is True) \
            and not bool(torch.all(hits))
        if not go:
            break
        logits = st.step(running_seq[:, :, cur - 1].reshape(-1), S0 + cur - 1)
    best_seq, best_idx = sequences[:, 0, :], beam_idx[:, 0, :]
    out_len = int(((best_idx + 1) != 0).sum(dim=1).max().item())
    return [list(map(int, r)) for r in best_seq[:, :out_len].cpu().tolist()]


HF_TOP_K = 50   # GenerationConfig default; text_decoder.py:131-144 never overrides it


def sampling_scores(logits: torch.Tensor, seqs: torch.Tensor, *, temperature: float, top_p: float, rep: float,
                    ngram: int, min_new: int, eos: int, top_k: int = HF_TOP_K) -> torch.Tensor:
    """The scores `_sample` draws from (HF generate with do_sample, text_decoder.py:131-144):
    processors (RepetitionPenalty -> NoRepeatNGram -> MinNewTokens) then warpers in HF's order
    (TemperatureLogitsWarper -> TopKLogitsWarper(50, the default the reference inherits) ->
    TopPLogitsWarper; min_tokens_to_keep 1, filter value -inf)."""
    sc = _processors(logits.float(), seqs, rep, ngram, min_new, eos)
    if temperature != 1.0:
        sc = sc / temperature
    if top_k:
        kth = torch.topk(sc, min(top_k, sc.shape[-1]), dim=-1).values[..., -1:]
        sc = sc.masked_fill(sc < kth, -float("inf"))
    if top_p < 1.0:
        sorted_logits, sorted_idx = torch.sort(sc, descending=False)
        cum = sorted_logits.softmax(dim=-1).cumsum(dim=-1)
        remove = cum <= (1 - top_p)
        remove[..., -1:] = False
        sc = sc.masked_fill(remove.scatter(1, sorted_idx, remove), -float("inf"))
    return sc


@torch.no_grad()
def sample(dec, prefix: torch.Tensor, prompt_ids: Sequence[int], *, temperature: float, top_p: float,
           max_new_tokens: int, min_new_tokens: int = 8, no_repeat_ngram_size: int = 3,
           repetition_penalty: float = 1.1, eos: int = 50256, seed: int = 0, top_k: int = HF_TOP_K,
           use_graph: bool = True) -> List[List[int]]:
    """HF `_sample` on the device (csrc/sample.hip through vcap_gpt2_sample: the greedy graph's
    processors, then Temperature -> TopK -> TopP and a Philox draw per row and step, one hipGraph,
    no host sync per token); rows cut where HF's stopping criteria end the batch."""
    from .model import GenConfig, trim_generated
    cfg = GenConfig(max_new_tokens, min_new_tokens, no_repeat_ngram_size, repetition_penalty, eos, eos, use_graph,
                    temperature=temperature, top_k=top_k, top_p=top_p, seed=seed)
    if not cfg.do_sample:
        raise ValueError("sampling needs temperature != 1 (HF do_sample rule, text_decoder.py:137)")
    return trim_generated(dec.generate_ids(prefix, list(prompt_ids), cfg), eos)
