"""roctx stage ranges for rocprofv3 (`--marker-trace`, `--kernel-rename`): the reference's NVTX ranges
ViT_Encoder / Cross_Modal_Alignment / GPT2_Decoder_Step (core/scripts/benchmark_baseline.py:31-41,
265-286; core/scripts/profile_nsight.py:24-34) on AMD's marker API.

Off by default: `range(name)` is a no-op context until `enable()` is called (bench.py --roctx), so
the timed region of a default run makes no roctx calls.  The ranges are host-side and bracket the
LAUNCH of a stage's work (the pipeline's launches are asynchronous); `rocprofv3 --kernel-rename`
names every kernel dispatched inside a range after it, which is how a profile attributes kernel time
to stages (tools/stage_profile.sh).  librocprofiler-sdk-roctx is the marker library rocprofv3
intercepts; it ships with ROCm, and without a profiler attached its calls return at once.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from typing import Optional

_lib: Optional[C.CDLL] = None
_enabled = False

VIT = "ViT_Encoder"
ALIGN = "Cross_Modal_Alignment"
DECODE = "GPT2_Decoder_Step"


def _load() -> C.CDLL:
    global _lib
    if _lib is None:
        last = None
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so"):
            try:
                lib = C.CDLL(name)
                break
            except OSError as e:
                last = e
        else:
            raise RuntimeError(f"roctx ranges asked for but librocprofiler-sdk-roctx is not loadable: {last}")
        lib.roctxRangePushA.argtypes, lib.roctxRangePushA.restype = [C.c_char_p], C.c_int
        lib.roctxRangePop.argtypes, lib.roctxRangePop.restype = [], C.c_int
        lib.roctxMarkA.argtypes, lib.roctxMarkA.restype = [C.c_char_p], None
        _lib = lib
    return _lib


def enable(on: bool = True) -> None:
    """Turn the stage ranges on (loads the marker library; raises if it is absent)."""
    global _enabled
    if on:
        _load()
    _enabled = bool(on)


def enabled() -> bool:
    return _enabled


@contextlib.contextmanager
def range(name: str):   # noqa: A001  (the roctx / NVTX vocabulary)
    if not _enabled:
        yield
        return
    lib = _load()
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    if _enabled:
        _load().roctxMarkA(name.encode())
