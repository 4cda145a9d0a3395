#!/bin/bash
# usage (GPU box): tools/bench_ab.sh <outdir> <steps> "<ENV=VAL ...>" "<ENV=VAL ...>" ...
# the default bench once per environment setting, interleaved twice, same box
out=$1; steps=$2; shift 2
mkdir -p $out
i=0
for rep in 1 2; do
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python bench.py --steps $steps --cpu-baseline-s 0 --host-e2e 0 --no-parity > $out/b$i.json 2> $out/b$i.err || exit 1
    python3 -c "
import json,sys;d=json.load(open('$out/b$i.json'))
print('$e', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'fc1', round(d['roofline']['avg_launch_ms']*1e3,1), 'attn', round(d['attention']['avg_launch_ms']*1e3,1))"
  done
done
