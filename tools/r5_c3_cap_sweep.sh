#!/bin/bash
# configs[3] decode grid cap sweep now that beam searches honour it (quick legs off, one box).
out=${1:-gpurun_out/r5c3cap}
mkdir -p $out
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
C3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 4"
for P in bf16 fp32; do
  for cap in 96 48 64 128 32 96; do
    tag="${P}_b$cap"
    timeout -k 10 400 python -u bench.py $C3 $quick --decode-blocks $cap --dec-precision $P > $out/$tag.json 2> $out/$tag.err || exit $?
    python3 -c "
import json
d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1])
print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,1) for k,v in d['stage_ms_p50'].items()})" | tee -a $out/summary.txt
  done
done
