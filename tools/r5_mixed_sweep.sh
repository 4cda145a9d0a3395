#!/bin/bash
# Schedule sweep for the token-exact mixed configuration (ViT bf16, decoder fp32), quick legs off.
out=${1:-gpurun_out/r5ms}
mkdir -p $out
Q="--steps 40 --warmup 5 --cpu-baseline-s 0 --no-parity --no-decode-alone --host-e2e 0 --strict-steps 0 --dec-precision fp32"
i=0
for ARGS in "" "--dec-lanes 3" "--reserve-cus 64" "--dec-lanes 3 --reserve-cus 48" "--decode-blocks 128" "--decode-blocks 0"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py $Q $ARGS > $out/m$i.json 2> $out/m$i.err || exit $?
  python3 -c "
import json; d=json.loads(open('$out/m$i.json').read().strip().splitlines()[-1])
print('[$ARGS]', round(d['value'],1), 'p50', round(d['p50_latency_ms'],2), {k: round(v,2) for k,v in d['stage_ms_p50'].items()})"
done
