"""Per-queue dependent-launch gaps in a rocprofv3 kernel trace of the pipelined bench: for every
hardware queue, kernels in start order, the gap from the previous kernel's end on that queue to this
kernel's start.  Splits the decode chain's time in the pipeline into kernel time and time between
kernels (compare tools/trace_gaps.py on the decode alone).

usage: python tools/queue_gaps.py <run_kernel_trace.csv>
"""
import csv
import statistics
import sys
from collections import defaultdict

DECODE = ("rows_gemv", "rows_gemm_lds", "decode_attention", "decode_finalize", "prefill_embed", "decode_init")


def main(path):
    per_q = defaultdict(list)
    with open(path) as f:
        rd = csv.DictReader(f)
        qcol = "Queue_Id" if "Queue_Id" in rd.fieldnames else "Stream_Id"
        for r in rd:
            per_q[r[qcol]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    print(f"{'queue':>6} {'kernels':>8} {'decode':>7} {'sum_dur_ms':>10} {'sum_gap_ms':>10} {'gap_p50_us':>10} "
          f"{'gap_p90_us':>10} {'dur_p50_us':>10}")
    for q, ks in sorted(per_q.items()):
        ks.sort()
        gaps, durs = [], []
        ndec = 0
        for i, (s, e, n) in enumerate(ks):
            is_dec = any(d in n for d in DECODE)
            ndec += is_dec
            if not is_dec:
                continue
            durs.append((e - s) / 1e3)
            if i > 0:
                g = (s - ks[i - 1][1]) / 1e3
                if 0 <= g < 200:  # a host-side gap between graph replays is not a dependent boundary
                    gaps.append(g)
        if not durs:
            print(f"{q:>6} {len(ks):8d} {0:7d}   (no decode kernels)")
            continue
        pct = lambda a, p: sorted(a)[min(len(a) - 1, int(p * len(a)))] if a else 0.0
        print(f"{q:>6} {len(ks):8d} {ndec:7d} {sum(durs) / 1e3:10.2f} {sum(gaps) / 1e3:10.2f} "
              f"{pct(gaps, 0.5):10.2f} {pct(gaps, 0.9):10.2f} {statistics.median(durs):10.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
