"""Build libvcap_hip.so in-tree with hipcc for gfx950 (no JIT, no torch extension).

The library is the product's only compute path: vcap._native loads it and raises if it is
missing.  `python -m vcap.build` (or __graft_entry__.build()) compiles each .hip source to an
object in parallel and links the shared library next to this file under _lib/.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent                      # video-caption-algorithm_amd/
CSRC = ROOT / "csrc"
INCLUDE = ROOT.parent / "include"
LIBDIR = PKG / "_lib"
LIB = LIBDIR / os.environ.get("VCAP_LIB_NAME", "libvcap_hip.so")
ARCH = os.environ.get("VCAP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         "-Wno-unused-result", f"-I{CSRC}", f"-I{INCLUDE}"] + os.environ.get("VCAP_EXTRA_FLAGS", "").split()


# per-file flags: the attention softmax never sees a NaN (masked keys are -inf), and without
# -fno-honor-nans every fmaxf of an MFMA result is preceded by a canonicalising v_max
FILE_FLAGS = {"vit_attention.hip": ["-fno-honor-nans"]}


def sources():
    return sorted(CSRC.glob("*.hip"))


def _digest() -> str:
    h = hashlib.sha256()
    for p in sources() + sorted(CSRC.glob("*.h")) + [INCLUDE / "vcap.h"]:
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(" ".join(FLAGS).encode())
    h.update(repr(sorted(FILE_FLAGS.items())).encode())
    return h.hexdigest()


def _compile(src: Path, obj: Path):
    cmd = [HIPCC, *FLAGS, *FILE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
    return obj


def build(force: bool = False, jobs: int | None = None) -> Path:
    LIBDIR.mkdir(parents=True, exist_ok=True)
    stamp = LIBDIR / (LIB.name + ".sha256")
    dig = _digest()
    if LIB.exists() and stamp.exists() and stamp.read_text() == dig and not force:
        return LIB
    objdir = LIBDIR / ("obj" + ("_" + LIB.stem if LIB.name != "libvcap_hip.so" else ""))
    objdir.mkdir(exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 1, len(sources()))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, objdir / (s.stem + ".o")), sources()))
    tmp = LIBDIR / (LIB.name + ".tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, LIB)
    stamp.write_text(dig)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
