"""Dependent-chain view of a rocprofv3 kernel trace: kernels in start order, each kernel's duration
and the gap from the previous kernel's end to its start (the dependent-launch boundary), summed per
kernel name over the window of launches whose name matches.  For the decode graph alone this splits
a token step into time inside kernels and time between them.

usage: python tools/trace_gaps.py <run_kernel_trace.csv> [name-substring ...]
"""
import csv
import statistics
import sys
from collections import defaultdict


def main(path, subs):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1), int(r["Grid_Size_Y"])))
    rows.sort()
    per = defaultdict(lambda: ([], []))
    prev_end = None
    tot_d = tot_g = 0.0
    for s, e, name, gx, gy in rows:
        if subs and not any(x in name for x in subs):
            prev_end = e
            continue
        d = (e - s) / 1e3
        g = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = e
        if g > 50:  # a host gap (between graph replays), not a dependent boundary
            continue
        key = (name[:90], gx, gy)
        per[key][0].append(d)
        per[key][1].append(g)
        tot_d += d
        tot_g += g
    print(f"{'launches':>8} {'dur_mean':>9} {'dur_min':>8} {'gap_mean':>9} {'gap_min':>8}  grid  kernel")
    for (name, gx, gy), (ds, gs) in sorted(per.items(), key=lambda kv: -sum(kv[1][0])):
        print(f"{len(ds):8d} {statistics.mean(ds):9.2f} {min(ds):8.2f} {statistics.mean(gs):9.2f} {min(gs):8.2f}  "
              f"{gx}x{gy}  {name}")
    print(f"# total in kernels {tot_d:.1f} us, between kernels {tot_g:.1f} us "
          f"(gaps {100 * tot_g / max(tot_d + tot_g, 1e-9):.1f} % of the chain)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
