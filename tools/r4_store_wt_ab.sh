#!/bin/bash
# fc1 output stores write-through (sc1 nt) vs nt: a variant library built aside (libvcap_wt.so,
# VCAP_GEMM_STORE_WT=1) against the product library, the GEMM alone and the pipelined bench.
out=${1:-gpurun_out/wt}
mkdir -p "$out"
wt="VCAP_LIB=$PWD/video-caption-algorithm_amd/vcap/_lib/libvcap_wt.so VCAP_GEMM_STORE_WT=1"
timeout -k 10 120 python -u tools/gemm_bench.py 50432 > "$out/gemm_0.txt" 2>&1 || exit $?
env $wt timeout -k 10 120 python -u tools/gemm_bench.py 50432 > "$out/gemm_1.txt" 2>&1 || exit $?
grep fc1 "$out/gemm_0.txt" | sed "s/^/nt /" | tee -a "$out/summary.txt"
grep fc1 "$out/gemm_1.txt" | sed "s/^/wt /" | tee -a "$out/summary.txt"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $quick > "$out/b_0_$i.json" 2> "$out/b_0_$i.err" || exit $?
  env $wt timeout -k 10 300 python -u bench.py $quick > "$out/b_1_$i.json" 2> "$out/b_1_$i.err" || exit $?
  for w in 0 1; do
    python3 -c "import json; d=json.loads(open('$out/b_${w}_$i.json').read().strip().splitlines()[-1]); print('wt=$w run $i', round(d['value'],1), 'fc1 us', round(d['roofline']['avg_launch_ms']*1e3,1))" | tee -a "$out/summary.txt"
  done
done
