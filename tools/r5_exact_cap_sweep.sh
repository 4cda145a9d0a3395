#!/bin/bash
# Token-exact configuration (bf16 ViT, fp32 decoder, configs[1] shape): decode grid cap sweep, quick legs off.
out=${1:-gpurun_out/r5excap}
mkdir -p $out
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for cap in 96 64 48 128 96; do
  tag="fp32dec_b$cap"
  timeout -k 10 400 python -u bench.py $quick --steps 40 --decode-blocks $cap --dec-precision fp32 > $out/$tag.json 2> $out/$tag.err || exit $?
  python3 -c "
import json
d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1])
print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,1) for k,v in d['stage_ms_p50'].items()})" | tee -a $out/summary.txt
done
