#!/bin/bash
# Decode lanes / decode confinement / hardware-queue sweep on one box (quick legs off, 60 timed
# batches of 8).  Each entry: "HWQ LANES RESERVE CONFINE".  usage: tools/r4_lanes_sweep.sh OUTDIR
out=${1:-gpurun_out/lanes}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for cfg in "4 2 32 0" "4 3 32 0" "8 3 32 0" "8 3 32 1" "8 4 48 1" "8 3 48 1" "8 4 64 1" "4 2 32 0"; do
  set -- $cfg
  tag="q$1_l$2_r$3_c$4"
  extra=""
  [ "$4" = 1 ] && extra="--confine-decode"
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python -u bench.py $quick --dec-lanes $2 --reserve-cus $3 $extra > "$out/$tag.json" 2> "$out/$tag.err" || exit $?
  python3 -c "import json; d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), 'stage', {k: round(v,2) for k, v in d['stage_ms_p50'].items()})" | tee -a "$out/summary.txt"
done
