"""The N-rank launch path the driver's multi-GPU runs take (`python bench.py --gpus N`, nccl): in a
fresh process on the GPU box, counting the GPUs (amdsmi) leaves HIP uninitialised, and the parent is
still uninitialised when it reaches spawn_ranks (one process per GPU, started before any
GPU call).  The spawn itself is replaced by a recorder: a one-GPU box cannot host the ranks."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]

SCRIPT = r"""
import json, sys
sys.argv = ["bench.py", "--gpus", "2"]
sys.path.insert(0, %r)
import bench, torch
n = bench._visible_gpus()                      # the real amdsmi count
after_count = torch.cuda.is_initialized()
args = bench.parse()
refused = bench.launch_check(args) if n < 2 else None   # a one-GPU box refuses --gpus 2 ...
seen = []
bench.spawn_ranks = lambda k: seen.append((k, torch.cuda.is_initialized())) or 0
bench._GPU_COUNT[0] = max(n, 2)                 # ... so pretend a second GPU to reach the spawn
rc = bench.launch_check(args)
print(json.dumps({"visible": n, "init_after_count": after_count, "refused": refused, "rc": rc, "spawn": seen,
                  "init_at_end": torch.cuda.is_initialized()}))
"""


def test_launcher_counts_gpus_without_initialising_hip():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "VCAP_BENCH_DIST_BACKEND")}
    r = subprocess.run([sys.executable, "-c", SCRIPT % str(ROOT)], env=env, capture_output=True, text=True,
                       timeout=120, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["visible"] >= 1
    assert d["init_after_count"] is False
    assert d["refused"] in (None, 2)
    assert d["rc"] == 0 and d["spawn"] == [[2, False]]
    assert d["init_at_end"] is False
