"""bench.py --gpus N launcher (BASELINE.json "1/2/4/8 GPU"): without torchrun, bench.py
starts the N ranks itself; under a launcher, N must equal WORLD_SIZE; N beyond the visible GPUs
is refused unless the gloo rehearsal is asked for.  CPU only: the refusals return before any GPU
call, and --dry-launch runs the rendezvous + one gloo all-gather of the ranks without GPU work."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

BENCH = Path(__file__).resolve().parents[1] / "bench.py"


def _run(args, **env):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "VCAP_BENCH_DIST_BACKEND")}
    e.update(env)
    return subprocess.run([sys.executable, str(BENCH), *args], env=e, capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("args,env,msg", [
    (["--gpus", "0"], {}, "--gpus must be >= 1"),
    (["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, "WORLD_SIZE=2"),
    (["--gpus", "2"], {}, "visible GPUs"),                      # no GPU here, no rehearsal env
    (["--gpus", "2"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, "visible GPUs"),
])
def test_refusals(args, env, msg):
    r = _run(args, **env)
    assert r.returncode == 2, (r.stdout, r.stderr)
    assert msg in r.stderr and not r.stdout.strip()


@pytest.mark.parametrize("n", [2, 4])
def test_self_launch_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--dry-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout                     # only rank 0 prints
    d = json.loads(lines[0])
    assert d["world_size"] == n and d["ranks"] == list(range(n))
    assert d["launcher"].startswith("bench.py --gpus")


def test_single_process_dry_launch():
    r = _run(["--gpus", "1", "--dry-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["world_size"] == 1


def test_failing_rank_status_is_returned(tmp_path):
    """Rank 1 dies at start-up (a sitecustomize on the children's path exits 3 when RANK == 1):
    the launcher stops rank 0, which would otherwise wait in the rendezvous, and returns 3."""
    (tmp_path / "sitecustomize.py").write_text(
        "import os\nif os.environ.get('RANK') == '1':\n    os._exit(3)\n")
    r = _run(["--gpus", "2", "--dry-launch"], PYTHONPATH=str(tmp_path))
    assert r.returncode == 3, (r.stdout, r.stderr[-2000:])
    assert "dry_launch" not in r.stdout


def test_gpu_count_never_falls_back_to_hip_init(tmp_path):
    """When amdsmi cannot count the GPUs, the launcher refuses instead of calling
    torch._C._cuda_getDeviceCount() (a HIP initialisation in the parent of the ranks): a sitecustomize
    makes the amdsmi count fail and the HIP count exit with status 7 if it is ever reached."""
    (tmp_path / "sitecustomize.py").write_text(
        "import os, torch\n"
        "torch.cuda._device_count_amdsmi = lambda: -1\n"
        "def _hip_count():\n    os._exit(7)\n"
        "torch._C._cuda_getDeviceCount = _hip_count\n")
    r = _run(["--gpus", "2"], PYTHONPATH=str(tmp_path))
    assert r.returncode == 2, (r.stdout, r.stderr[-2000:])
    assert "amdsmi could not count" in r.stderr
