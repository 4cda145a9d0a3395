#!/bin/bash
# Round 5 bench lines on one box: the token-exact fp32 configuration, the reference's own precision
# split (ViT bf16 + decoder fp32), and the driver's default command.  usage: tools/r5_lines.sh <outdir>
out=${1:-gpurun_out/r5lines}
mkdir -p $out
timeout -k 10 400 python -u bench.py --precision fp32 --steps 20 --warmup 5 > $out/fp32.json 2> $out/fp32.err || exit $?
timeout -k 10 400 python -u bench.py --dec-precision fp32 --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bf16.json 2> $out/bf16.err || exit $?
for f in fp32 mixed bf16; do python3 -c "
import json,sys
d=json.loads(open('$out/$f.json').read().strip().splitlines()[-1])
p=d.get('parity') or {}; o=d.get('oracle_parity') or {}
print('$f', round(d['value'],1), 'p50', round(d['p50_latency_ms'],2), 'dtype', d['dtype'], 'step_us', round(d['decode_roofline']['step_us'],1),
      'parity', p.get('captions_identical'), '/', p.get('captions'), 'oracle', o.get('captions_identical'), '/', o.get('captions'),
      'roof', round(d['roofline']['frac'],3))"; done
