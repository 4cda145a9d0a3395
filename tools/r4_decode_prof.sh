#!/bin/bash
# rocprofv3 kernel trace of the launch-chain decode alone (tools/persist_time.py, persistent off):
# per-kernel average durations of one token step.  usage (GPU box): tools/r4_decode_prof.sh <outdir> [lm_stream 0|1]
out=${1:-gpurun_out/decprof}; lm=${2:-1}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
cd /tmp && export TMPDIR=/tmp
VCAP_LM_STREAM=$lm PERSIST_GS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/trace -o run -- python3 $root/tools/persist_time.py 8 > $root/$out/time.log 2>&1 || exit $?
s=$(find $root/$out/trace -name "run_kernel_stats.csv" | head -1)
cp $s $root/$out/kernel_stats.csv
python3 - "$root/$out/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:90]:90s} calls {r["Calls"]:>6s} avg {float(r["AverageNs"])/1e3:8.2f} us')
PY
