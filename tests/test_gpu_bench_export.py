"""bench.py --export-csv / --export-json end to end on the GPU (the reference harness's files:
core/scripts/benchmark_baseline.py:394-454): one batch size -> per-iteration CSV + summary JSON with
one row per timed batch; a --batch-sizes sweep -> the batch-size comparison CSV + per-batch JSON."""
import csv
import json
import subprocess
import sys
from pathlib import Path

import pytest

from vcap import report

pytestmark = pytest.mark.gpu
BENCH = Path(__file__).resolve().parents[1] / "bench.py"
QUICK = ["--warmup", "1", "--cpu-baseline-s", "0", "--no-parity", "--no-decode-alone", "--host-e2e", "0",
         "--strict-steps", "0"]


def _bench(args):
    r = subprocess.run([sys.executable, str(BENCH), *QUICK, *args], capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def test_iteration_exports(tmp_path):
    c, j = tmp_path / "it.csv", tmp_path / "s.json"
    line = _bench(["--steps", "6", "--export-csv", str(c), "--export-json", str(j)])
    with open(c) as fh:
        rows = list(csv.DictReader(fh))
    assert list(rows[0].keys()) == report.ITERATION_FIELDS and len(rows) == 6
    assert all(float(r["iteration_ms"]) > float(r["vit_encoder_ms"]) > 0 for r in rows)
    assert all(r["caption_preview"].startswith("ids ") for r in rows)
    d = json.loads(j.read_text())
    assert d["summary"]["iterations"] == 6 and d["summary"]["batch_size"] == 8
    assert d["summary"]["generated_tokens"]["count"] == 6 * 8
    assert abs(d["summary"]["End_to_end_Latency"]["p50_ms"] - line["p50_latency_ms"]) < 1e-6
    assert d["bench_line"]["value"] == line["value"]


def test_batch_size_comparison_exports(tmp_path):
    c, j = tmp_path / "cmp.csv", tmp_path / "cmp.json"
    _bench(["--steps", "4", "--batch-sizes", "2,8", "--sweep-steps", "4", "--export-csv", str(c),
            "--export-json", str(j)])
    with open(c) as fh:
        rows = list(csv.DictReader(fh))
    assert list(rows[0].keys()) == report.COMPARISON_FIELDS
    assert [int(r["batch_size"]) for r in rows] == [2, 8] and all(r["status"] == "ok" for r in rows)
    d = json.loads(j.read_text())
    assert sorted(d["per_batch_summary"]) == ["2", "8"] and len(d["per_batch_iterations"]["8"]) == 4
