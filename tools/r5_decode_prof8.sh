#!/bin/bash
# Per-kernel split of the decode step alone at B = 8 rows (uncapped grids), bf16 and fp32 decoders.
out=${1:-gpurun_out/r5dp8}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
cd /tmp && export TMPDIR=/tmp
for P in bf16 fp32; do
  B=8 PREC=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/$P -o run -- python3 $root/tools/decode_step_time.py > $root/$out/$P.txt 2>&1 || exit $?
  f=$(find $root/$out/$P -name "run_kernel_trace.csv" | head -1)
  python3 $root/tools/kernel_trace_summary.py $f > $root/$out/${P}_split.txt || exit $?
done
echo done
