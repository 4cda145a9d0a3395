"""One line per kernel from the tools/qa_pmc.sh passes: wave-cycle split (parked on waits, issue-stalled,
LDS-stalled, issuing), MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8
XCDs) as tools/pmc_report.py prices it, L2 hit rate, FETCH_SIZE x 2 (gfx950 correction) per launch.
usage: python tools/qa_pmc_summary.py <qa_pmc outdir>"""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if not any(s in name for s in ("gemm256", "vit_attention", "qkv_attention")):
            continue
        acc[name[:80]][r["Counter_Name"]].append(float(r["Counter_Value"]))


def avg(c, k):
    v = c.get(k, [])
    return sum(v) / len(v) if v else float("nan")


for name, c in acc.items():
    wc = avg(c, "SQ_WAVE_CYCLES")
    print(f"{name}: waits {avg(c, 'SQ_WAIT_ANY') / wc:.2f}, issue-stalled {avg(c, 'SQ_WAIT_INST_ANY') / wc:.2f} "
          f"(LDS {avg(c, 'SQ_WAIT_INST_LDS') / wc:.3f}), issuing {avg(c, 'SQ_ACTIVE_INST_ANY') / wc:.2f}; "
          f"MFMA util {avg(c, 'SQ_VALU_MFMA_BUSY_CYCLES') / (1024 * avg(c, 'GRBM_GUI_ACTIVE') / 8):.3f}; "
          f"L2 hit {avg(c, 'TCC_HIT_sum') / (avg(c, 'TCC_HIT_sum') + avg(c, 'TCC_MISS_sum')):.3f}; "
          f"FETCH x2 {2 * avg(c, 'FETCH_SIZE') / 1e3:.0f} MB")
