"""Live per-launch kernel timing (vcap_probe_*): HIP events recorded around every launch of a probed
encode site ("vit.fc1", "vit.attention", ...) on the stream it is launched on, with the launch's
row count, so bench.py prices each launch with its own FLOP / byte count."""
from __future__ import annotations

import ctypes as C
from collections import defaultdict
from typing import Dict, List, Tuple

from . import _native as N


def enable(site: str, max_launches: int) -> None:
    N.check(N.lib().vcap_probe_enable(site.encode(), int(max_launches)), f"probe enable {site}")


def read(site: str, cap: int) -> List[Tuple[float, int]]:
    """[(ms, rows)] of every launch recorded since enable(); disables the site."""
    ms = (C.c_float * max(cap, 1))()
    rows = (C.c_int * max(cap, 1))()
    n = C.c_int()
    N.check(N.lib().vcap_probe_read_launches(site.encode(), ms, rows, int(cap), C.byref(n)), f"probe read {site}")
    return [(float(ms[i]), int(rows[i])) for i in range(n.value)]


def by_rows(launches: List[Tuple[float, int]]) -> Dict[int, List[float]]:
    """Launch times grouped by their row count (one population per encode batch size)."""
    out: Dict[int, List[float]] = defaultdict(list)
    for ms, r in launches:
        out[r].append(ms)
    return dict(out)
