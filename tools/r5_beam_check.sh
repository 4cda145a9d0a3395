#!/bin/bash
# Beam-step rework check: the beam / decode GPU tests, then the configs[3] step alone (fp32 / bf16,
# B = 8 and 4 sequences x 4 beams) and its per-kernel split.
out=${1:-gpurun_out/r5bc}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_search.py tests/test_gpu_large.py tests/test_gpu_decode_tiles.py tests/test_gpu_lm_screen.py > $root/$out/tests.txt 2>&1 || { tail -30 $root/$out/tests.txt; exit 1; }
tail -3 $root/$out/tests.txt
for P in fp32 bf16; do
  for B in 8 4; do
    B=$B BEAMS=4 GPT2=gpt2-medium PREC=$P timeout -k 10 200 python3 tools/decode_step_time.py >> $root/$out/steps.txt 2>&1 || exit $?
  done
done
cat $root/$out/steps.txt
cd /tmp && export TMPDIR=/tmp
for P in fp32 bf16; do
  B=8 BEAMS=4 GPT2=gpt2-medium PREC=$P timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/$P -o run -- python3 $root/tools/decode_step_time.py > $root/$out/$P.txt 2>&1 || exit $?
  f=$(find $root/$out/$P -name "run_kernel_trace.csv" | head -1)
  python3 $root/tools/kernel_trace_summary.py $f > $root/$out/${P}_split.txt || exit $?
done
echo done
