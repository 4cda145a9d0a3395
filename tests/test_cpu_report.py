"""bench.py --export-csv / --export-json (vcap/report.py) against the reference harness's export
shapes: core/scripts/benchmark_baseline.py:394-454 (CSV columns, JSON payload), :114-157 (stats),
:352-385 (summary), :548-586 (comparison row)."""
import ast
import csv
import json
import math
from pathlib import Path

import pytest

from vcap import report

REF = Path("/root/reference/core/scripts/benchmark_baseline.py")

# the reference's lists, restated (benchmark_baseline.py:396-415 and :426-443)
REF_ITERATION = ["iter_index", "batch_size", "iteration_ms", "throughput_samples_per_s", "caption_preview",
                 "generated_tokens_mean", "preprocess_cuda_ms", "preprocess_host_ms", "preprocess_peak_mb",
                 "vit_encoder_ms", "vit_encoder_peak_mb", "cross_modal_alignment_ms",
                 "cross_modal_alignment_peak_mb", "gpt2_decoder_ms", "gpt2_decoder_peak_mb",
                 "gpt2_token_step_mean_ms", "gpt2_token_step_max_ms", "max_memory_allocated_mb"]
REF_COMPARISON = ["batch_size", "status", "warmup", "iters", "end_to_end_mean_ms", "end_to_end_std_ms",
                  "preprocess_mean_ms", "preprocess_std_ms", "vit_mean_ms", "vit_std_ms", "gpt2_mean_ms",
                  "gpt2_std_ms", "throughput_mean_samples_per_s", "throughput_std_samples_per_s",
                  "throughput_from_mean_latency_samples_per_s", "max_memory_allocated_mb"]


def test_columns_match_reference_lists():
    assert report.ITERATION_FIELDS == REF_ITERATION
    assert report.COMPARISON_FIELDS == REF_COMPARISON


@pytest.mark.skipif(not REF.exists(), reason="reference tree not mounted (build container only)")
def test_columns_match_reference_source():
    """The same lists read out of the reference file's AST (study of its text, nothing executed)."""
    tree = ast.parse(REF.read_text(encoding="utf-8-sig"))   # the file starts with a BOM
    found = {}
    for fn in tree.body:
        if isinstance(fn, ast.FunctionDef) and fn.name in ("export_iteration_csv", "export_bs_comparison_csv"):
            for node in ast.walk(fn):
                if isinstance(node, ast.Assign) and getattr(node.targets[0], "id", "") == "fieldnames":
                    found[fn.name] = [e.value for e in node.value.elts]
    assert found["export_iteration_csv"] == report.ITERATION_FIELDS
    assert found["export_bs_comparison_csv"] == report.COMPARISON_FIELDS


def test_percentile_and_stats_follow_reference():
    assert report.percentile([], 0.5) != report.percentile([], 0.5)   # nan
    assert report.percentile([3.0], 0.99) == 3.0
    v = [1.0, 2.0, 3.0, 4.0]
    assert math.isclose(report.percentile(v, 0.99), 3.97)          # (n-1)*q = 2.97 -> 3 + 0.97
    st = report.stats_dict(v)
    assert st["count"] == 4 and st["mean_ms"] == 2.5 and math.isclose(st["std_ms"], 1.118033988749895)
    assert st["max_ms"] == 4.0 and st["min_ms"] == 1.0 and st["p50_ms"] == 2.5
    assert report.stats_dict([])["mean_ms"] is None
    t = report.throughput_stats_dict([10.0, 20.0])
    assert t["mean_samples_per_s"] == 15.0 and t["std_samples_per_s"] == 5.0


def _rows():
    return report.iteration_rows(8, [20.0, 30.0], [12.0, 13.0], [8.0, 17.0], [[5, 24] * 4, [9] * 8],
                                 ["ids 1 2", "ids 3"], 0.25, 1024.0)


def test_iteration_csv_and_summary_json(tmp_path):
    rows = _rows()
    p = tmp_path / "sub" / "it.csv"
    report.export_iteration_csv(str(p), rows)
    with open(p) as fh:
        r = list(csv.DictReader(fh))
    assert list(r[0].keys()) == REF_ITERATION
    assert [x["iter_index"] for x in r] == ["1", "2"]
    assert float(r[0]["throughput_samples_per_s"]) == 8 / 0.020
    s = report.build_summary(rows, 8)
    for k in ("status", "batch_size", "Preprocess_Latency", "Preprocess_CUDA_Latency", "ViT_Latency",
              "Cross_Modal_Alignment", "GPT2_Latency", "GPT2_token_step", "End_to_end_Latency", "Throughput",
              "generated_tokens", "peak_memory_mb", "caption_preview", "iterations"):
        assert k in s, k                                             # benchmark_baseline.py:360-385
    assert s["End_to_end_Latency"]["mean_ms"] == 25.0
    assert s["Throughput"]["from_mean_latency_samples_per_s"] == 8 / 0.025
    assert s["generated_tokens"]["count"] == 16 and s["generated_tokens"]["max"] == 24
    j = tmp_path / "s.json"
    report.export_summary_json(str(j), {"summary": s, "iterations": rows})
    assert json.loads(j.read_text())["summary"]["iterations"] == 2


def test_comparison_csv(tmp_path):
    s = report.build_summary(_rows(), 8)
    row = report.comparison_row(s, 4, 2)
    assert list(row.keys()) == REF_COMPARISON
    assert row["end_to_end_mean_ms"] == 25.0 and row["vit_mean_ms"] == 12.5 and row["gpt2_mean_ms"] == 12.5
    bad = report.comparison_row({"status": "OOM", "batch_size": 64, "peak_memory_mb": {}}, 4, 2)
    assert bad["end_to_end_mean_ms"] is None and bad["status"] == "OOM"
    p = tmp_path / "cmp.csv"
    report.export_bs_comparison_csv(str(p), [row, bad])
    with open(p) as fh:
        r = list(csv.DictReader(fh))
    assert list(r[0].keys()) == REF_COMPARISON and len(r) == 2
