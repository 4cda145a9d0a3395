"""Where a decode token step's time goes, from the in-kernel clock stamps of the diagnostic build
(tools/build_stamps.py -> VCAP_LIB=.../libvcap_stamps.so).  Runs the B-row HF-greedy decode graph
alone, then for every launch of the replay reports (median over its workgroups, thread 0 of wave 0):
  start  = first workgroup entry - previous launch's last epilogue issue (the dependent boundary as
           the CUs see it, plus the last stores draining)
  act    = entry -> activation operand landed (PRO_LN: LayerNorm tile written, barrier passed;
           PRO_DIRECT: the last A fragment's load returned)
  wgt    = -> weight stream landed (the wave's last weight fragment returned)
  mfma   = -> MFMAs retired (split-K partials written to LDS)
  red    = -> split-K reduction barrier passed
  epi    = -> epilogue issued
  skew   = last workgroup entry - first workgroup entry
  span   = first entry -> last epilogue issue
grouped by the launch's role within a layer.  Units: microseconds (100 MHz clock)."""
import ctypes as C
import os
import statistics
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "video-caption-algorithm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vcap import _native as N  # noqa: E402
from vcap import configs, weights  # noqa: E402
from vcap.model import GenConfig, HipGPT2Decoder  # noqa: E402

ROLE = {0x0: "c_attn(LN+QKV)", 0x2: "c_fc(LN+GELU)", 0x1: "c_proj(+res)", 0x3: "lm_head(LN+proc)"}


def role(tag):
    if tag == 0xA000:
        return "attention"
    if tag == 0xC000:   # act = ln_f tile ready, wgt = 1st column group, mfma = 2nd, red = the rest, epi = partials
        return "lm_head stream (act=LN, wgt=group0, mfma=group1, red=rest, epi=partials)"
    epi, pro, nsl = (tag >> 8) & 0xF, (tag >> 4) & 0xF, (tag >> 12) & 0xFF
    name = {0: "c_attn(LN+QKV)", 2: "c_fc(LN+GELU)", 1: "c_proj(+res)", 3: "lm_head(LN+proc)"}.get(epi, f"epi{epi}")
    return f"{name} nsl{nsl}" + (" half" if (tag >> 24) & 1 else "")


def main():
    name = os.environ.get("GPT2", "gpt2")
    ga = configs.gpt2_arch(name)
    dev = torch.device("cuda:0")
    prec = os.environ.get("PREC", "bf16")
    dec = HipGPT2Decoder(weights.synthetic_gpt2(1, ga), ga, prec, dev)
    lib = N.lib()
    lib.vcap_diag_stamps.restype = C.c_int
    lib.vcap_diag_stamps.argtypes = [C.c_void_p, C.c_int]
    B = int(os.environ.get("B", "8"))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        pre = torch.randn(B, 4, ga.n_embd, device=dev) * 0.1
        cfg = GenConfig(24, 8, 3, 1.1, ga.eos_token_id, ga.eos_token_id, True)
        cfg.max_blocks = int(os.environ.get("CAP", "0"))
        for _ in range(3):
            dec.generate_ids(pre, [ga.bos_token_id], cfg)
        torch.cuda.synchronize()
        lib.vcap_diag_stamps(None, 0)
        dec.generate_ids(pre, [ga.bos_token_id], cfg)
        torch.cuda.synchronize()
    buf = np.zeros((1 << 18, 8), dtype=np.uint64)
    n = lib.vcap_diag_stamps(buf.ctypes.data, buf.shape[0])
    rec = buf[:n].astype(np.int64)
    rec = rec[np.argsort(rec[:, 2], kind="stable")]
    # split into launches: consecutive records (by entry time) with the same tag and grid
    launches, cur = [], []
    for r in rec:
        key = (int(r[0]), int(r[1]) >> 20 & 0xFFFFF)
        if cur and (key != cur[0][0] or r[2] > max(x[1][7] for x in cur) + 200):
            launches.append(cur)
            cur = []
        cur.append((key, r))
    if cur:
        launches.append(cur)
    per = defaultdict(lambda: defaultdict(list))
    prev_end = None
    tot = defaultdict(float)
    for L in launches:
        rs = np.array([r for _, r in L])
        t0 = rs[:, 2].min()
        end = rs[:, 7].max()
        key = role(L[0][0][0]) + f" grid{L[0][0][1]}"
        d = per[key]
        if prev_end is not None and 0 <= t0 - prev_end < 10000:
            d["start"].append((t0 - prev_end) / 100)
            tot["start"] += (t0 - prev_end) / 100
        for c, (i, j) in {"act": (2, 3), "wgt": (3, 4), "mfma": (4, 5), "red": (5, 6), "epi": (6, 7)}.items():
            d[c].append(np.median(rs[:, j] - rs[:, i]) / 100)
            tot[c] += np.median(rs[:, j] - rs[:, i]) / 100
        d["skew"].append((rs[:, 2].max() - t0) / 100)
        d["span"].append((end - t0) / 100)
        tot["span"] += (end - t0) / 100
        prev_end = end
    print(f"{name} {prec} B={B} cap={cfg.max_blocks}: {len(launches)} launches, {n} workgroup records")
    cols = ["start", "act", "wgt", "mfma", "red", "epi", "skew", "span"]
    print(f"{'launches':>8} " + " ".join(f"{c:>6}" for c in cols) + "  role")
    for key, d in sorted(per.items(), key=lambda kv: -sum(kv[1]["span"])):
        print(f"{len(d['span']):8d} " + " ".join(f"{statistics.median(d[c]) if d[c] else 0:6.2f}" for c in cols)
              + f"  {key}")
    print(f"# sum over the replay ({len(launches)} launches): spans {tot['span']:.0f} us, starts {tot['start']:.0f} us; "
          "median workgroup phases " + ", ".join(f"{c} {tot[c]:.0f}" for c in ("act", "wgt", "mfma", "red", "epi")) + " us")


if __name__ == "__main__":
    main()
