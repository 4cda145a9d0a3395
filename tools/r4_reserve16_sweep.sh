#!/bin/bash
# CU reservation for the unpaired 16-video batches (bf16 and the fp8 configs[4] shape), quick legs off.
out=${1:-gpurun_out/res16}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for cfg in "bf16 0" "bf16 32" "fp8 0" "fp8 32" "bf16 16" "fp8 16"; do
  set -- $cfg
  tag="$1_b16_r$2"
  timeout -k 10 300 python -u bench.py $quick --precision $1 --batch 16 --steps 30 --reserve-cus $2 > "$out/$tag.json" 2> "$out/$tag.err" || exit $?
  python3 -c "import json; d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,2) for k, v in d['stage_ms_p50'].items()})" | tee -a "$out/summary.txt"
done
