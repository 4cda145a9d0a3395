#!/bin/bash
# bench.py schedule sweep (no CPU baseline / parity / decode-alone legs):
#   "lanes group reserve blocks [confine]"
out=${1:-gpurun_out/sweep}; shift; mkdir -p $out
for cfg in "$@"; do
  set -- $cfg
  extra=""; tag=""
  if [ "$5" = "c" ]; then extra="--confine-decode"; tag="_c"; fi
  f=$out/l$1_g$2_r$3_b$4$tag.json
  timeout -k 10 120 python bench.py --steps 40 --warmup 4 --dec-lanes $1 --dec-group $2 --reserve-cus $3 \
    --decode-blocks $4 $extra --cpu-baseline-s 0 --no-parity --no-decode-alone --host-e2e 0 > $f 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('lanes $1 group $2 reserve $3 blocks $4 $5:', round(d['value'],1), 'captions/s', 'p50', round(d['p50_latency_ms'],1), 'ms', 'fc1', round(d['roofline']['avg_launch_ms']*1e3,1), 'us')"
done
