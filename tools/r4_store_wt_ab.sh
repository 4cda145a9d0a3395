#!/bin/bash
# fc1 output stores write-through (VCAP_GEMM_STORE_WT=1: sc1 nt) vs nt, alone and in the bench.
out=${1:-gpurun_out/wt}
mkdir -p "$out"
for w in 0 1; do
  VCAP_GEMM_STORE_WT=$w timeout -k 10 120 python -u tools/gemm_bench.py 50432 > "$out/gemm_$w.txt" 2>&1 || exit $?
  grep fc1 "$out/gemm_$w.txt" | sed "s/^/wt=$w /" | tee -a "$out/summary.txt"
done
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for i in 1 2; do
  for w in 0 1; do
    VCAP_GEMM_STORE_WT=$w timeout -k 10 300 python -u bench.py $quick > "$out/b_${w}_$i.json" 2> "$out/b_${w}_$i.err" || exit $?
    python3 -c "import json; d=json.loads(open('$out/b_${w}_$i.json').read().strip().splitlines()[-1]); print('wt=$w run $i', round(d['value'],1), 'fc1 us', round(d['roofline']['avg_launch_ms']*1e3,1))" | tee -a "$out/summary.txt"
  done
done
