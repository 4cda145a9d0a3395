#!/bin/bash
# configs[3] (ViT-L/14 + GPT-2-medium, 32 frames, beam 4, max_new 40): bf16 and the reference's
# precision split (ViT bf16 + decoder fp32); fp8 configs[4] shape with an fp32 decoder.
out=${1:-gpurun_out/r5c3}
mkdir -p $out
C3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 4"
timeout -k 10 500 python -u bench.py $C3 --dec-precision fp32 > $out/c3_mixed.json 2> $out/c3_mixed.err || exit $?
timeout -k 10 500 python -u bench.py $C3 > $out/c3_bf16.json 2> $out/c3_bf16.err || exit $?
timeout -k 10 400 python -u bench.py --precision fp8 --batch 16 --steps 30 --dec-precision fp32 > $out/fp8_mixed.json 2> $out/fp8_mixed.err || exit $?
for f in c3_mixed c3_bf16 fp8_mixed; do python3 -c "
import json
d=json.loads(open('$out/$f.json').read().strip().splitlines()[-1])
p=d.get('parity') or {}
print('$f', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), d['dtype'], 'step', round(d['decode_roofline']['step_us'],1), {k: p.get(k) for k in ('captions','captions_identical','hypotheses_identical','max_fp32_score_deficit','best_identical')})"; done
