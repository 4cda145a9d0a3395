"""Summarise a rocprofv3 kernel trace (run_kernel_trace.csv) per (kernel, grid size): launches and
mean / min / max duration, so one launch population (e.g. the 16-video fc1 GEMM of the timed
region, 50432 rows -> its own grid) reads directly against bench.py's live per-launch probe.

usage: python tools/kernel_trace_summary.py <run_kernel_trace.csv> [name-substring ...] > summary.txt
"""
import csv
import statistics
import sys
from collections import defaultdict


def main(path, subs):
    pops = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if subs and not any(s in name for s in subs):
                continue
            grid = (int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1), int(r["Grid_Size_Y"]),
                    int(r["Grid_Size_Z"]))
            pops[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = sorted(pops.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'total_us':>10} {'launches':>8} {'mean_us':>9} {'min_us':>9} {'max_us':>9}  workgroups  kernel")
    for (name, grid), d in rows:
        short = name if len(name) < 110 else name[:107] + "..."
        print(f"{sum(d):10.1f} {len(d):8d} {statistics.mean(d):9.2f} {min(d):9.2f} {max(d):9.2f}  "
              f"{grid[0]}x{grid[1]}x{grid[2]}  {short}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
