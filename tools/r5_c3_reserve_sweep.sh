#!/bin/bash
# configs[3] encode-stream CU reservation (the L/14 GEMMs' tile rounds: 4112 fc1 tiles are 18.4 rounds on
# 224 CUs, 17.1 on 240), bf16 and fp32 decoder, quick legs off, one box.
out=${1:-gpurun_out/r5c3r}
mkdir -p $out
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
C3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 4"
for P in bf16 fp32; do
  for r in 32 16 24 8 32; do
    tag="${P}_r$r"
    timeout -k 10 400 python -u bench.py $C3 $quick --reserve-cus $r --dec-precision $P > $out/$tag.json 2> $out/$tag.err || exit $?
    python3 -c "
import json
d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1])
print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,1) for k,v in d['stage_ms_p50'].items()})" | tee -a $out/summary.txt
  done
done
