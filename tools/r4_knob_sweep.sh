#!/bin/bash
# Default-schedule knob sweep on one box (quick legs off, 60 timed batches of 8): encode-stream CU
# reservation and the decode GEMV grid cap.  Entry: "RESERVE BLOCKS".  usage: tools/r4_knob_sweep.sh OUTDIR
out=${1:-gpurun_out/knobs}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for cfg in "32 96" "24 96" "40 96" "16 96" "32 64" "32 128" "32 80" "32 96"; do
  set -- $cfg
  tag="r$1_b$2"
  timeout -k 10 300 python -u bench.py $quick --reserve-cus $1 --decode-blocks $2 > "$out/$tag.json" 2> "$out/$tag.err" || exit $?
  python3 -c "import json; d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,2) for k, v in d['stage_ms_p50'].items()})" | tee -a "$out/summary.txt"
done
