#!/bin/bash
# strict-batch schedule (one 8-video encode + one 8-row decode per batch) over the encode stream's
# CU reservation, as the main timed run (quick legs off).  usage: tools/r4_strict_sweep.sh OUTDIR
out=${1:-gpurun_out/strict}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for r in 0 16 32 48 0; do
  tag="eg1_dg1_r$r"
  timeout -k 10 300 python -u bench.py $quick --enc-group 1 --dec-group 1 --reserve-cus $r > "$out/$tag.json" 2> "$out/$tag.err" || exit $?
  python3 -c "import json; d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,2) for k, v in d['stage_ms_p50'].items()})" | tee -a "$out/summary.txt"
done
