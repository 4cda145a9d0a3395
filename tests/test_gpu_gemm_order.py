"""The 256x256 GEMM's tile order (row-major, or the column groups fc1 runs in by default:
csrc/gemm256.hip GemmEpi.colgroup) changes which workgroup computes a tile and when, never a tile's
arithmetic: the fc1-shaped GEMM's output is bit-identical under every order.  One child process per
order, since the dispatcher reads VCAP_GEMM_COLGROUP once per process."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
HERE = Path(__file__).resolve().parent


def _digest(colgroup, rows):
    env = dict(os.environ)
    if colgroup is None:
        env.pop("VCAP_GEMM_COLGROUP", None)
    else:
        env["VCAP_GEMM_COLGROUP"] = str(colgroup)
    r = subprocess.run([sys.executable, str(HERE / "gemm_order_worker.py"), str(rows)], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout.strip().splitlines()[-1]


@pytest.mark.parametrize("rows", [2560, 50432 - 17])
def test_fc1_tile_orders_bit_identical(rows):
    ref = _digest(0, rows)                                    # row-major
    assert _digest(None, rows) == ref                         # the default (groups of 6)
    assert _digest(4, rows) == ref
    assert _digest(2, rows) == ref
