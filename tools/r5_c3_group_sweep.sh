#!/bin/bash
# configs[3] bf16 encode / decode grouping after the late changes (quick legs off, one box).
out=${1:-gpurun_out/r5c3g}
mkdir -p $out
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
C3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 4"
for cfg in "2 2 3" "1 2 3" "1 1 3" "2 2 2" "1 1 2" "2 2 3"; do
  set -- $cfg
  tag="eg$1_dg$2_l$3"
  timeout -k 10 400 python -u bench.py $C3 $quick --enc-group $1 --dec-group $2 --dec-lanes $3 > $out/$tag.json 2> $out/$tag.err || exit $?
  python3 -c "
import json
d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1])
print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,1) for k,v in d['stage_ms_p50'].items()})" | tee -a $out/summary.txt
done
