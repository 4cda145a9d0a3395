#!/bin/bash
# Confined-decode sweep (decode streams masked to the reserved CUs) over the decode GEMV grid cap,
# one box, quick legs off.  Entry: "LANES RESERVE BLOCKS".  usage: tools/r4_confine_sweep.sh OUTDIR
out=${1:-gpurun_out/confine}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
timeout -k 10 300 python -u bench.py $quick > "$out/default.json" 2> "$out/default.err" || exit $?
python3 -c "import json; d=json.loads(open('$out/default.json').read().strip().splitlines()[-1]); print('default', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,2) for k, v in d['stage_ms_p50'].items()})" | tee -a "$out/summary.txt"
for cfg in "3 32 32" "3 32 64" "3 40 40" "3 48 48" "2 48 48"; do
  set -- $cfg
  tag="l$1_r$2_b$3"
  timeout -k 10 300 python -u bench.py $quick --confine-decode --dec-lanes $1 --reserve-cus $2 --decode-blocks $3 > "$out/$tag.json" 2> "$out/$tag.err" || exit $?
  python3 -c "import json; d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,2) for k, v in d['stage_ms_p50'].items()})" | tee -a "$out/summary.txt"
done
