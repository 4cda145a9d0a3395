#!/bin/bash
# QKV column groups (VCAP_GEMM_COLGROUP_QKV 0 / 3) under the default schedule, interleaved.
out=${1:-gpurun_out/qkvcg}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for w in 0 3 0 3; do
  VCAP_GEMM_COLGROUP_QKV=$w timeout -k 10 300 python -u bench.py $quick > "$out/b_$w.json" 2> "$out/b_$w.err" || exit $?
  python3 -c "import json; d=json.loads(open('$out/b_$w.json').read().strip().splitlines()[-1]); print('qkv colgroup=$w', round(d['value'],1), {k: round(v,2) for k, v in d['stage_ms_p50'].items()})" | tee -a "$out/summary.txt"
done
