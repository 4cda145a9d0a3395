#!/bin/bash
# Per-kernel split of the configs[3] beam step alone (GPT-2-medium, 4 beams, device search graph):
# B = 8 sequences (the pipeline's 2-batch decode group = 32 rows), fp32 and bf16 decoders.
out=${1:-gpurun_out/r5bm}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
cd /tmp && export TMPDIR=/tmp
for P in fp32 bf16; do
  B=8 BEAMS=4 GPT2=gpt2-medium PREC=$P timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/$P -o run -- python3 $root/tools/decode_step_time.py > $root/$out/$P.txt 2>&1 || exit $?
  f=$(find $root/$out/$P -name "run_kernel_trace.csv" | head -1)
  python3 $root/tools/kernel_trace_summary.py $f > $root/$out/${P}_split.txt || exit $?
done
echo done
