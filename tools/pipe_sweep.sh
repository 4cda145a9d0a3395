#!/bin/bash
# bench.py schedule sweep (no CPU baseline / parity / decode-alone legs): lanes x group x reserve
out=${1:-gpurun_out/sweep}; mkdir -p $out
for cfg in "2 1 32" "1 2 32" "2 2 32" "1 2 64" "2 2 64" "1 2 0" "2 2 0"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --steps 30 --warmup 4 --dec-lanes $1 --dec-group $2 --reserve-cus $3 \
    --cpu-baseline-s 0 --no-parity --no-decode-alone --host-e2e 0 > $out/l$1_g$2_r$3.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('$out/l$1_g$2_r$3.json').read().strip().splitlines()[-1]); print('lanes $1 group $2 reserve $3:', round(d['value'],1), 'captions/s', 'p50', round(d['p50_latency_ms'],1), 'ms', 'fc1', round(d['roofline']['avg_launch_ms']*1e3,1), 'us')"
done
