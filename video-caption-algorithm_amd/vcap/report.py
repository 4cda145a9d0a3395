"""The reference benchmark harness's exports for bench.py (`--export-csv`, `--export-json`).

Same columns and payload shapes as `core/scripts/benchmark_baseline.py`: the per-iteration CSV
(`export_iteration_csv`, :394-421), the batch-size comparison CSV (`export_bs_comparison_csv`,
:424-448), the summary JSON (`export_summary_json` :451-454 with the payloads of :683-737) and
the statistics behind them (`percentile` / `stats_dict` / `throughput_stats_dict`, :114-157;
`build_summary` :352-385; `build_comparison_row` :548-586).  Host-side bookkeeping only.

What a column means here: an "iteration" is one timed batch of the pipelined schedule
(encode start -> ids on the device); frames are already resident in HBM, so the preprocessing
columns are 0; the prefix LN-scale + mapper (the reference's Cross_Modal_Alignment stage) run
inside the fused encode launch sequence, so that column is 0 and its time is in vit_encoder_ms;
the per-token step columns come from the decode-step-alone measurement (one replayed hipGraph
has no per-token host timing)."""
from __future__ import annotations

import csv
import json
import math
import statistics
from pathlib import Path
from typing import Dict, List, Optional, Sequence

# core/scripts/benchmark_baseline.py:396-415
ITERATION_FIELDS = [
    "iter_index", "batch_size", "iteration_ms", "throughput_samples_per_s", "caption_preview",
    "generated_tokens_mean", "preprocess_cuda_ms", "preprocess_host_ms", "preprocess_peak_mb",
    "vit_encoder_ms", "vit_encoder_peak_mb", "cross_modal_alignment_ms", "cross_modal_alignment_peak_mb",
    "gpt2_decoder_ms", "gpt2_decoder_peak_mb", "gpt2_token_step_mean_ms", "gpt2_token_step_max_ms",
    "max_memory_allocated_mb",
]
# core/scripts/benchmark_baseline.py:426-443
COMPARISON_FIELDS = [
    "batch_size", "status", "warmup", "iters", "end_to_end_mean_ms", "end_to_end_std_ms",
    "preprocess_mean_ms", "preprocess_std_ms", "vit_mean_ms", "vit_std_ms", "gpt2_mean_ms", "gpt2_std_ms",
    "throughput_mean_samples_per_s", "throughput_std_samples_per_s",
    "throughput_from_mean_latency_samples_per_s", "max_memory_allocated_mb",
]


def percentile(values: Sequence[float], q: float) -> float:
    """Linear interpolation between closest ranks (benchmark_baseline.py:114-126)."""
    if not values:
        return float("nan")
    v = sorted(values)
    if len(v) == 1:
        return v[0]
    r = (len(v) - 1) * q
    lo, hi = math.floor(r), math.ceil(r)
    return v[lo] if lo == hi else v[lo] * (1.0 - (r - lo)) + v[hi] * (r - lo)


def stats_dict(values: Sequence[float]) -> Dict[str, Optional[float]]:
    """benchmark_baseline.py:129-139 (population std), plus p50 (the north-star metric's)."""
    if not values:
        return {"count": 0, "mean_ms": None, "std_ms": None, "p99_ms": None, "max_ms": None, "min_ms": None,
                "p50_ms": None}
    return {"count": len(values), "mean_ms": statistics.mean(values),
            "std_ms": statistics.pstdev(values) if len(values) > 1 else 0.0,
            "p99_ms": percentile(values, 0.99), "max_ms": max(values), "min_ms": min(values),
            "p50_ms": percentile(values, 0.5)}


def throughput_stats_dict(values: Sequence[float]) -> Dict[str, Optional[float]]:
    """benchmark_baseline.py:142-157."""
    if not values:
        return {"count": 0, "mean_samples_per_s": None, "std_samples_per_s": None,
                "max_samples_per_s": None, "min_samples_per_s": None}
    return {"count": len(values), "mean_samples_per_s": statistics.mean(values),
            "std_samples_per_s": statistics.pstdev(values) if len(values) > 1 else 0.0,
            "max_samples_per_s": max(values), "min_samples_per_s": min(values)}


def iteration_rows(batch: int, lat_ms: Sequence[float], vit_ms: Sequence[float], dec_ms: Sequence[float],
                   gen_lens: Sequence[Sequence[int]], previews: Sequence[str], token_step_ms: Optional[float],
                   max_mem_mb: float) -> List[dict]:
    """One row per timed batch (run_one_iteration's return dict, benchmark_baseline.py:296-316)."""
    rows = []
    for k, (lt, vt, dt) in enumerate(zip(lat_ms, vit_ms, dec_ms)):
        lens = gen_lens[k] if k < len(gen_lens) else []
        rows.append({
            "batch_size": batch, "iteration_ms": lt, "throughput_samples_per_s": batch / (lt / 1e3),
            "caption_preview": previews[k] if k < len(previews) else "",
            "generated_tokens": list(lens),
            "generated_tokens_mean": statistics.mean(lens) if lens else 0.0,
            "preprocess_cuda_ms": 0.0, "preprocess_host_ms": 0.0, "preprocess_peak_mb": max_mem_mb,
            "vit_encoder_ms": vt, "vit_encoder_peak_mb": max_mem_mb,
            "cross_modal_alignment_ms": 0.0, "cross_modal_alignment_peak_mb": max_mem_mb,
            "gpt2_decoder_ms": dt, "gpt2_decoder_peak_mb": max_mem_mb,
            "gpt2_token_step_mean_ms": token_step_ms if token_step_ms is not None else 0.0,
            "gpt2_token_step_max_ms": token_step_ms if token_step_ms is not None else 0.0,
            "max_memory_allocated_mb": max_mem_mb,
        })
    return rows


def build_summary(rows: Sequence[dict], batch: int, status: str = "ok") -> dict:
    """benchmark_baseline.py:352-385 over the iteration rows."""
    lat = [r["iteration_ms"] for r in rows]
    tput = [r["throughput_samples_per_s"] for r in rows]
    e2e = stats_dict(lat)
    lens = [n for r in rows for n in r.get("generated_tokens", [])]   # per-caption lengths
    tok = [r["gpt2_token_step_mean_ms"] for r in rows]
    mem = max((r["max_memory_allocated_mb"] for r in rows), default=None)
    return {
        "status": status, "batch_size": batch,
        "Preprocess_Latency": stats_dict([r["preprocess_host_ms"] for r in rows]),
        "Preprocess_CUDA_Latency": stats_dict([r["preprocess_cuda_ms"] for r in rows]),
        "ViT_Latency": stats_dict([r["vit_encoder_ms"] for r in rows]),
        "Cross_Modal_Alignment": stats_dict([r["cross_modal_alignment_ms"] for r in rows]),
        "GPT2_Latency": stats_dict([r["gpt2_decoder_ms"] for r in rows]),
        "GPT2_token_step": stats_dict(tok),
        "End_to_end_Latency": e2e,
        "Throughput": {**throughput_stats_dict(tput),
                       "from_mean_latency_samples_per_s": batch / (e2e["mean_ms"] / 1e3) if e2e["mean_ms"] else None},
        "generated_tokens": {"count": len(lens), "mean": statistics.mean(lens) if lens else None,
                             "max": max(lens) if lens else None},
        "peak_memory_mb": {"max_memory_allocated_mb": mem},
        "caption_preview": rows[-1]["caption_preview"] if rows else "",
        "iterations": len(rows),
    }


def comparison_row(summary: dict, warmup: int, iters: int) -> dict:
    """benchmark_baseline.py:548-586."""
    ok = summary.get("status") == "ok"

    def g(stage, key):
        return summary[stage][key] if ok else None
    return {"batch_size": summary["batch_size"], "status": summary["status"], "warmup": warmup, "iters": iters,
            "end_to_end_mean_ms": g("End_to_end_Latency", "mean_ms"), "end_to_end_std_ms": g("End_to_end_Latency", "std_ms"),
            "preprocess_mean_ms": g("Preprocess_Latency", "mean_ms"), "preprocess_std_ms": g("Preprocess_Latency", "std_ms"),
            "vit_mean_ms": g("ViT_Latency", "mean_ms"), "vit_std_ms": g("ViT_Latency", "std_ms"),
            "gpt2_mean_ms": g("GPT2_Latency", "mean_ms"), "gpt2_std_ms": g("GPT2_Latency", "std_ms"),
            "throughput_mean_samples_per_s": g("Throughput", "mean_samples_per_s"),
            "throughput_std_samples_per_s": g("Throughput", "std_samples_per_s"),
            "throughput_from_mean_latency_samples_per_s": g("Throughput", "from_mean_latency_samples_per_s"),
            "max_memory_allocated_mb": summary["peak_memory_mb"]["max_memory_allocated_mb"] if ok else None}


def _parent(path: str) -> None:
    Path(path).parent.mkdir(parents=True, exist_ok=True)


def export_iteration_csv(path: str, rows: Sequence[dict]) -> None:
    """benchmark_baseline.py:394-421 (iter_index from 1)."""
    _parent(path)
    with open(path, "w", newline="", encoding="utf-8") as fh:
        w = csv.DictWriter(fh, fieldnames=ITERATION_FIELDS)
        w.writeheader()
        for i, row in enumerate(rows, start=1):
            w.writerow({"iter_index": i, **{k: row.get(k) for k in ITERATION_FIELDS if k != "iter_index"}})


def export_bs_comparison_csv(path: str, rows: Sequence[dict]) -> None:
    """benchmark_baseline.py:424-448."""
    _parent(path)
    with open(path, "w", newline="", encoding="utf-8") as fh:
        w = csv.DictWriter(fh, fieldnames=COMPARISON_FIELDS)
        w.writeheader()
        for row in rows:
            w.writerow({k: row.get(k) for k in COMPARISON_FIELDS})


def export_summary_json(path: str, payload: dict) -> None:
    """benchmark_baseline.py:451-454."""
    _parent(path)
    with open(path, "w", encoding="utf-8") as fh:
        json.dump(payload, fh, ensure_ascii=False, indent=2)
