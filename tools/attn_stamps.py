"""ViT attention workgroup timeline from the stamp build (tools/build_stamps.py): one launch at the
benchmark shape (BT frames x 197 tokens x 12 heads, bf16), then per workgroup the K/V/Q load phase
(entry -> all landed + barrier), the compute + store-issue phase, which CU it ran on and how many
workgroups overlapped on that CU.  Units: microseconds (100 MHz clock)."""
import ctypes as C
import os
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402

BT, NT, H = int(os.environ.get("BT", "128")), 197, 12
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(BT * NT, 3 * H * 64, generator=g, device=dev).to(torch.bfloat16)
out = torch.empty(BT * NT, H * 64, device=dev, dtype=torch.bfloat16)
s = torch.cuda.current_stream().cuda_stream
lib = N.lib()
lib.vcap_diag_stamps_attn.restype = C.c_int
lib.vcap_diag_stamps_attn.argtypes = [C.c_void_p, C.c_int]
for _ in range(5):
    N.check(lib.vcap_vit_attention(N.DT_BF16, qkv.data_ptr(), out.data_ptr(), BT, NT, H, s), "attn")
torch.cuda.synchronize()
lib.vcap_diag_stamps_attn(None, 0)
N.check(lib.vcap_vit_attention(N.DT_BF16, qkv.data_ptr(), out.data_ptr(), BT, NT, H, s), "attn")
torch.cuda.synchronize()
buf = np.zeros((1 << 18, 8), dtype=np.uint64)
n = lib.vcap_diag_stamps_attn(buf.ctypes.data, buf.shape[0])
r = buf[:n].astype(np.int64)
t0, t1, t2 = r[:, 2], r[:, 3], r[:, 4]
base = t0.min()
hw = r[:, 7] & 0xFFFFFFFF
xcc = (r[:, 7] >> 32) & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 0x1
se = (hw >> 13) & 0x7
unit = xcc * 1000 + se * 100 + sh * 10 + cu
load, comp = (t1 - t0) / 100, (t2 - t1) / 100
q = lambda a: " / ".join(f"{np.percentile(a, p):.2f}" for p in (10, 50, 90))
print(f"attention BT={BT}: {n} workgroups, kernel span {(t2.max() - base) / 100:.1f} us "
      f"(first entry -> last store issue)")
print(f"load phase (p10/p50/p90) {q(load)} us; compute+store phase {q(comp)} us")
per = defaultdict(list)
for i in range(n):
    per[int(unit[i])].append((t0[i], t2[i]))
conc, busy = [], []
for u, iv in per.items():
    iv.sort()
    busy.append(sum(b - a for a, b in iv) / 100)
    ev = sorted([(a, 1) for a, _ in iv] + [(b, -1) for _, b in iv])
    c = m = 0
    for _, d in ev:
        c += d
        m = max(m, c)
    conc.append(m)
print(f"distinct CUs {len(per)}, workgroups per CU p50 {np.median([len(v) for v in per.values()]):.0f}, "
      f"max concurrent per CU p50 {np.median(conc):.0f}, per-CU summed WG lifetime p50 {np.median(busy):.1f} us")
# entry-time histogram: are the workgroups in lockstep rounds?
edges = np.linspace(0, (t2.max() - base) / 100, 11)
hist, _ = np.histogram((t0 - base) / 100, bins=edges)
print("entries per tenth of the span:", " ".join(str(h) for h in hist))
hist, _ = np.histogram((t1 - base) / 100, bins=edges)
print("loads landed per tenth:       ", " ".join(str(h) for h in hist))
