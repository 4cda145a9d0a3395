"""Per-kernel averages of the counters tools/pmc.sh collected: python tools/pmc_summary.py <outdir> [name-filter]."""
import csv
import glob
import sys
from collections import defaultdict

out = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{out}/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if flt and flt not in name:
            continue
        acc[name[:110]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, ctrs in acc.items():
    print(name)
    for c, v in sorted(ctrs.items()):
        print(f"    {c:28s} n={len(v):5d} avg={sum(v) / len(v):.4g}")
