#!/bin/bash
# Hardware queues per process (GPU_MAX_HW_QUEUES 4 = the box default, 8, 16) under the default
# schedule, interleaved, quick legs off.  usage: tools/r4_hwq_ab.sh OUTDIR
out=${1:-gpurun_out/hwq}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for i in 1 2; do
  for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py $quick > "$out/q${q}_$i.json" 2> "$out/q${q}_$i.err" || exit $?
    python3 -c "import json; d=json.loads(open('$out/q${q}_$i.json').read().strip().splitlines()[-1]); print('hwq=$q run $i', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,2) for k, v in d['stage_ms_p50'].items()})" | tee -a "$out/summary.txt"
  done
done
