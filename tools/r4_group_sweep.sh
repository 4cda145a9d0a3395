#!/bin/bash
# Pipeline grouping sweep on one box (quick legs off, 60 timed batches of 8): encode / decode group
# sizes and the encode stream's CU reservation.  usage: tools/r4_group_sweep.sh OUTDIR
out=${1:-gpurun_out/groups}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for cfg in "2 2 32" "3 3 32" "3 3 0" "3 3 64" "4 4 32" "2 2 32"; do
  set -- $cfg
  tag="dg$1_eg$2_r$3"
  timeout -k 10 300 python -u bench.py $quick --dec-group $1 --enc-group $2 --reserve-cus $3 > "$out/$tag.json" 2> "$out/$tag.err" || exit $?
  python3 -c "import json; d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), 'fc1 us', round(d['roofline']['avg_launch_ms']*1e3,1))" | tee -a "$out/summary.txt"
done
