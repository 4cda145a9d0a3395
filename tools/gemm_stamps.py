"""Where a 256x256 GEMM launch spends its time, per workgroup (diagnostic build only).

Needs a library built with -DVCAP_GEMM_STAMPS (python -m vcap.build with
VCAP_LIB_NAME=gemm_stamps.so VCAP_EXTRA_FLAGS=-DVCAP_GEMM_STAMPS), loaded through VCAP_LIB.  Runs
each ViT GEMM shape at M rows on the 256x256 kernel (policy 2), then reads wave 0's 100 MHz
timestamps of every workgroup: entry, first K-tile landed, K loop done, epilogue stores issued,
stores complete.  Prints the launch span, phase medians, the per-round timeline and the gap a CU
sits idle between one workgroup's end and the next one's start.
"""
import ctypes as C
import statistics
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 50432
dev = torch.device("cuda:0")
lib = N.lib()
s = torch.cuda.current_stream().cuda_stream
import os
RESERVE = int(os.environ.get("RESERVE", "0"))  # run on a stream CU-masked off RESERVE CUs (the bench's encode stream)
if RESERVE:
    h = C.c_void_p()
    N.check(lib.vcap_stream_create_cu_reserved(RESERVE, C.byref(h)), "stream")
    s = h.value
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*shape, scale=1.0, dtype=torch.bfloat16):
    return (torch.rand(*shape, generator=g, device=dev) * 2 - 1).mul_(scale).to(dtype)


shapes = {"qkv": (2304, 768, False, 0, False), "proj": (768, 768, True, 0, True),
          "fc1": (3072, 768, False, 1, False), "fc2": (768, 3072, True, 0, True)}
stamps_fn = getattr(lib, "vcap_diag_gemm_stamps")
stamps_fn.restype = C.c_int
stamps_fn.argtypes = [C.c_void_p, C.c_long]
lib.vcap_set_gemm_policy(2)
for name, (n, k, f32, act, res) in shapes.items():
    A, W = rnd(M, k), rnd(n, k, scale=0.05)
    b = rnd(n, scale=0.1, dtype=torch.float32)
    Cm = torch.zeros(M, n, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
    odt = N.DT_F32 if f32 else N.DT_BF16

    def run():
        N.check(lib.vcap_gemm(N.DT_BF16, odt, A.data_ptr(), k, W.data_ptr(), k, Cm.data_ptr(), n, M, n, k,
                              b.data_ptr(), act, Cm.data_ptr() if res else None, n if res else 0, 1 if res else 0,
                              0, 0, 0, 0, s), name)
    for _ in range(20):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    e1.synchronize()
    ev_us = e0.elapsed_time(e1) * 1e3
    tiles = ((M + 255) // 256) * ((n + 255) // 256)
    buf = np.zeros(8192 * 8, dtype=np.uint64)
    assert stamps_fn(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(8192, 8)[:tiles].astype(np.int64)
    t0 = st[:, 0].min()
    ent, lan, klp, iss, don = [(st[:, i] - t0) / 100.0 for i in range(5)]  # us
    span = don.max()
    print(f"== {name} M={M} N={n} K={k}: {tiles} tiles, event {ev_us:.1f} us, stamp span {span:.1f} us "
          f"(last entry {ent.max():.1f}, last K-loop end {klp.max():.1f})")
    med = lambda x: statistics.median(x.tolist())  # noqa: E731
    print(f"   per WG median: prologue {med(lan - ent):.2f}  K-loop {med(klp - lan):.2f}  epilogue issue "
          f"{med(iss - klp):.2f}  store drain {med(don - iss):.2f}  total {med(don - ent):.2f} us")
    print(f"   per WG p90:    prologue {np.percentile(lan - ent, 90):.2f}  K-loop {np.percentile(klp - lan, 90):.2f}"
          f"  epilogue issue {np.percentile(iss - klp, 90):.2f}  store drain {np.percentile(don - iss, 90):.2f}")
    order = np.argsort(ent)
    ncu = len({(int(v) >> 32, (int(v) >> 8) & 0xFF) for v in st[:, 5]})
    for r in range(0, tiles, 256):
        idx = order[r:r + 256]
        print(f"   round {r // 256}: {len(idx)} WGs entry {ent[idx].min():7.1f}..{ent[idx].max():7.1f}  "
              f"K-loop end med {med(klp[idx]):7.1f}  done med {med(don[idx]):7.1f} max {don[idx].max():7.1f}")
    # idle gap per CU: next workgroup's entry - previous workgroup's store completion / epilogue issue
    per_cu = defaultdict(list)
    for i in range(tiles):
        per_cu[(int(st[i, 5]) >> 32, (int(st[i, 5]) >> 8) & 0xFF)].append(i)
    gaps_done, gaps_iss = [], []
    for lst in per_cu.values():
        lst.sort(key=lambda i: ent[i])
        for a, b2 in zip(lst, lst[1:]):
            gaps_done.append(ent[b2] - don[a])
            gaps_iss.append(ent[b2] - iss[a])
    xcc = (st[:, 5] >> 32).astype(np.int64)
    bids = np.arange(tiles)
    for mod in (7, 8):
        same = np.mean([len(set(xcc[bids % mod == r].tolist())) == 1 for r in range(mod)])
        print(f"   bid % {mod}: fraction of residues whose workgroups all ran on one XCC: {same:.2f}")
    print(f"   XCCs used: {sorted(set(xcc.tolist()))}; first 16 bids -> XCC {xcc[:16].tolist()}")
    if gaps_done:
        print(f"   CUs seen {ncu}; gap next-entry minus prev stores-done: median {statistics.median(gaps_done):.2f} us; "
              f"minus prev epilogue-issued: median {statistics.median(gaps_iss):.2f} us")
lib.vcap_set_gemm_policy(0)
