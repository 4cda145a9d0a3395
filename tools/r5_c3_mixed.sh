#!/bin/bash
# configs[3] with the reference's precision split (decoder fp32), one line.
out=${1:-gpurun_out/r5c3m}
mkdir -p $out
C3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 4"
timeout -k 10 500 python -u bench.py $C3 --dec-precision fp32 > $out/c3_mixed.json 2> $out/c3_mixed.err || exit $?
python3 -c "
import json
d=json.loads(open('$out/c3_mixed.json').read().strip().splitlines()[-1])
p=d.get('parity') or {}
print('c3_mixed', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), d['stage_ms_p50'], 'step', round(d['decode_roofline']['step_us'],1), {k: p.get(k) for k in ('hypotheses_identical','max_score_deficit')})"
