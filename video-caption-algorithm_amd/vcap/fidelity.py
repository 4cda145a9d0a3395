"""Fidelity evidence for the reduced-precision paths (bf16 decode, bf16 / MXFP8 encode) against the
fp32 parity mode, which is token-identical to the reference's own generate() on the golden inputs
(tests/test_gpu_parity.py, tests/test_gpu_search.py).

A reduced-precision greedy decode can legitimately leave the reference's path only where the
reference's processed top-2 gap is smaller than the reduced path's logit error: before the first
such near-tie every argmax is the same.  `greedy_divergence` measures both quantities on the same
inputs - the fp32 decode's raw logits along its own tokens, and the reduced decoder TEACHER-FORCED
along those tokens (vcap_gpt2_forward_embeds) - and explains every divergent caption by the fp32
margin at its first divergent step.  It also returns the leading-token agreement those margins
guarantee (`guaranteed_lead`): a floor derived from the near-tie statistics, not from a measured
agreement.

Beam search (presets precise / detailed) keeps several hypotheses, so its evidence is a score
comparison instead: `hypothesis_scores` rescores any token sequence exactly as HF `_beam_search`
ranks finished hypotheses (text_decoder.py:131-144: log_softmax -> RepetitionPenalty ->
NoRepeatNGram -> MinNewTokens, summed over the generated tokens, / length ** length_penalty)
under the fp32 decoder, so a reduced-precision search's choice is priced against the reference's.

Processor semantics: vcap.search._processors (HF order; history = generated tokens only, because
the reference generates from inputs_embeds).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .model import GenConfig, HipGPT2Decoder
from .search import _processors


def _lm(dec: HipGPT2Decoder):
    from .caption import HipGPT2LMHead, _WTE
    return HipGPT2LMHead(dec, dec.arch, _WTE(dec.wte))


@torch.no_grad()
def teacher_forced_logits(dec: HipGPT2Decoder, prefix: torch.Tensor, prompt_ids: Sequence[int],
                          tokens: torch.Tensor, steps: int) -> torch.Tensor:
    """Raw logits [steps, rows, V] of `dec` fed prefix [rows, P, E] + the prompt, then tokens[:, s]
    after step s (the decoder's own wte rows, as its generate() feeds them)."""
    dev = prefix.device
    lm = _lm(dec)
    ids = torch.tensor(list(prompt_ids), dtype=torch.long, device=dev)
    x = torch.cat([prefix.float(), lm.transformer.wte(ids)[None].expand(prefix.shape[0], -1, -1)], 1)
    out = lm(inputs_embeds=x, use_cache=True)
    res = torch.empty(steps, prefix.shape[0], dec.arch.vocab, dtype=torch.float32, device=dev)
    tok = tokens.to(dev).long()
    for s in range(steps):
        res[s] = out.logits[:, -1, :]
        if s + 1 < steps:
            out = lm(inputs_embeds=lm.transformer.wte(tok[:, s])[:, None, :], past_key_values=out.past_key_values)
    return res


def _decided_steps(ids: np.ndarray, eos: int) -> np.ndarray:
    """Per row: number of steps whose token was an argmax decision (up to and including the first
    EOS; later steps are forced padding)."""
    L = ids.shape[1]
    out = np.full(ids.shape[0], L, dtype=np.int64)
    for b, row in enumerate(ids):
        hit = np.nonzero(row == eos)[0]
        if hit.size:
            out[b] = hit[0] + 1
    return out


@torch.no_grad()
def greedy_divergence(test_ids, ref_ids, ref_logits: torch.Tensor, test_tf_logits: torch.Tensor,
                      cfg: GenConfig) -> Dict:
    """Explain each caption where `test_ids` leaves `ref_ids` (both [B, L] greedy ids, HF processors
    per cfg).  ref_logits: fp32 raw logits [L, B, V] along ref_ids; test_tf_logits: the tested
    precision's raw logits teacher-forced along ref_ids.  Returns per-step error bounds, one record
    per divergent caption, and the leading-token agreement the margins guarantee at the measured
    error."""
    test_ids, ref_ids = np.asarray(test_ids), np.asarray(ref_ids)
    B, L = ref_ids.shape
    eos = int(cfg.eos_token_id)
    dev = ref_logits.device
    hist = torch.from_numpy(ref_ids.astype(np.int64)).to(dev)
    decided = _decided_steps(ref_ids, eos)
    raw_err, proc_err = [], []
    margins = np.full((L, B), np.inf)         # processed top-2 gap of the fp32 path at each decided step
    recs: List[Dict] = []
    first_div = np.array([next((s for s in range(L) if test_ids[b, s] != ref_ids[b, s]), L) for b in range(B)])
    for s in range(L):
        live = torch.from_numpy(decided > s).to(dev)
        r, t = ref_logits[s].double(), test_tf_logits[s].double()
        raw_err.append(float(((r - t).abs().amax(-1) * live).max()))
        pr = _processors(r, hist[:, :s], cfg.repetition_penalty, cfg.no_repeat_ngram_size, cfg.min_new_tokens, eos)
        pt = _processors(t, hist[:, :s], cfg.repetition_penalty, cfg.no_repeat_ngram_size, cfg.min_new_tokens, eos)
        fin = torch.isfinite(pr) & torch.isfinite(pt)
        d = torch.where(fin, (pr - pt).abs(), torch.zeros_like(pr)).amax(-1)
        proc_err.append(float((d * live).max()))
        top = torch.topk(pr, 2, dim=-1).values
        gap = (top[:, 0] - top[:, 1]).cpu().numpy()
        margins[s] = np.where(decided > s, gap, np.inf)
        for b in np.nonzero(first_div == s)[0]:
            if s >= decided[b]:
                continue
            a, c = int(ref_ids[b, s]), int(test_ids[b, s])
            recs.append({"caption": int(b), "step": int(s), "ref_token": a, "test_token": c,
                         "fp32_margin": float(pr[b, a] - pr[b, c]), "fp32_top2_gap": float(gap[b]),
                         "test_err_at_pair": float((pt[b, a] - pr[b, a]).abs() + (pt[b, c] - pr[b, c]).abs()),
                         "test_prefers_its_token": bool(pt[b, c] >= pt[b, a])})
    tol = max(proc_err)
    # before the first decided step whose fp32 top-2 gap is below 2 x the measured processed error,
    # every argmax of the tested path equals the reference's (|error| <= tol on both tokens)
    guard = np.array([next((s for s in range(int(decided[b])) if margins[s, b] <= 2 * tol), L) for b in range(B)])
    lead = np.array([next((s for s in range(L) if test_ids[b, s] != ref_ids[b, s]), L) for b in range(B)])
    return {"captions": int(B), "steps": int(L),
            "captions_identical": int(sum(bool(np.array_equal(test_ids[b], ref_ids[b])) for b in range(B))),
            "leading_token_agreement": float(np.mean(lead / L)),
            "position_agreement": float((test_ids == ref_ids).mean()),
            "max_raw_logit_err": max(raw_err), "max_processed_err": tol,
            "raw_logit_err_per_step": [round(x, 5) for x in raw_err],
            "divergences": recs,
            "every_divergence_within_error": all(r["fp32_margin"] <= r["test_err_at_pair"] + 1e-9 for r in recs),
            "guaranteed_lead": float(np.mean(guard / L)),
            "lead_at_least_guaranteed": bool(np.all(lead >= guard)),
            "fp32_top2_gap_quantiles": [float(q) for q in np.quantile(margins[np.isfinite(margins)], [0.0, 0.01, 0.1, 0.5])]}


@torch.no_grad()
def hypothesis_scores(dec: HipGPT2Decoder, prefix: torch.Tensor, prompt_ids: Sequence[int],
                      seqs: Sequence[Sequence[int]], cfg: GenConfig) -> List[float]:
    """HF beam-search score of each token sequence (row i continues prefix[i]): the sum over its
    generated tokens (up to and including the first EOS) of log_softmax -> RepetitionPenalty ->
    NoRepeatNGram -> MinNewTokens, divided by length ** length_penalty."""
    eos = int(cfg.eos_token_id)
    lens = []
    for s in seqs:
        s = [int(t) for t in s]
        lens.append(s.index(eos) + 1 if eos in s else len(s))
    L = max(lens)
    tok = torch.full((len(seqs), L), eos, dtype=torch.long)
    for i, s in enumerate(seqs):
        tok[i, :lens[i]] = torch.tensor([int(t) for t in s[:lens[i]]])
    tok = tok.to(prefix.device)
    logits = teacher_forced_logits(dec, prefix, prompt_ids, tok, L)
    total = torch.zeros(len(seqs), dtype=torch.float64, device=prefix.device)
    ln = torch.tensor(lens, device=prefix.device)
    for s in range(L):
        lp = F.log_softmax(logits[s].double(), dim=-1)
        lp = _processors(lp, tok[:, :s], cfg.repetition_penalty, cfg.no_repeat_ngram_size, cfg.min_new_tokens, eos)
        total += torch.where(ln > s, lp.gather(1, tok[:, s:s + 1])[:, 0], torch.zeros_like(total))
    return (total / ln.double() ** float(cfg.length_penalty)).cpu().tolist()


@torch.no_grad()
def beam_divergence(dec32: HipGPT2Decoder, prefix32: torch.Tensor, prompt_ids: Sequence[int],
                    test_seqs, ref_seqs, cfg: GenConfig, tol: Optional[float] = None) -> Dict:
    """Price a reduced-precision beam search's hypotheses under the fp32 decoder: for each sequence
    the fp32 score of the test's best hypothesis against the fp32 search's best (the reference's
    choice).  A search with per-token score error <= e can only swap hypotheses whose fp32 scores
    differ by about 2e; `score_deficit` is that difference."""
    tnorm = [list(map(int, r)) for r in test_seqs]
    rnorm = [list(map(int, r)) for r in ref_seqs]
    st = hypothesis_scores(dec32, prefix32, prompt_ids, tnorm, cfg)
    sr = hypothesis_scores(dec32, prefix32, prompt_ids, rnorm, cfg)
    eos = int(cfg.eos_token_id)

    def trim(r):
        return r[:r.index(eos) + 1] if eos in r else r
    same = [trim(a) == trim(b) for a, b in zip(tnorm, rnorm)]
    deficit = [float(b - a) for a, b in zip(st, sr)]
    out = {"sequences": len(rnorm), "hypotheses_identical": int(sum(same)),
           "fp32_score_of_test_best": st, "fp32_score_of_ref_best": sr, "score_deficit": deficit,
           "max_score_deficit": max(deficit) if deficit else 0.0}
    if tol is not None:
        out["deficit_tol"] = tol
        out["within_tol"] = bool(max(deficit) <= tol) if deficit else True
    return out
