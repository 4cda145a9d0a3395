#!/bin/bash
# usage (GPU box): tools/bench_envargs_ab.sh <outdir> "<ENV=V ...>|<bench args>" ...
# bench.py once per (environment, arguments) pair, interleaved twice, same box
out=$1; shift
mkdir -p $out
i=0
for rep in 1 2; do
  for spec in "$@"; do
    i=$((i+1))
    e=${spec%%|*}; a=${spec#*|}
    env $e timeout -k 10 300 python bench.py --cpu-baseline-s 0 --host-e2e 0 --no-parity --no-decode-alone $a > $out/b$i.json 2> $out/b$i.err || exit 1
    python3 -c "
import json;d=json.load(open('$out/b$i.json'))
print('$spec |', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'p50', round(d['p50_latency_ms'],1), {k: round(v,2) for k,v in d['stage_ms_p50'].items()})"
  done
done
