#!/bin/bash
# usage (GPU box): tools/bench_ab.sh <outdir> <lib A> <lib B> [rounds] [bench args...]
# alternate bench.py runs on two library builds ('-' = in-tree) on the same box
set -e
out=$1; a=$2; b=$3; rounds=${4:-2}; shift 4 || true
mkdir -p $out
for r in $(seq 1 $rounds); do
  for lib in $a $b; do
    tag=$(basename $lib .so); [ "$lib" = "-" ] && tag=intree
    if [ "$lib" = "-" ]; then unset VCAP_LIB; else export VCAP_LIB=$(cd "$(dirname $lib)" && pwd)/$(basename $lib); fi
    timeout -k 10 240 python bench.py --steps 30 --warmup 4 --cpu-baseline-s 0 --host-e2e 0 "$@" > $out/${tag}_$r.json 2> $out/${tag}_$r.err
    python -c "
import json,sys; d=json.loads(open('$out/${tag}_$r.json').read().strip().splitlines()[-1])
print('$tag', $r, round(d['value'],1), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms_p50'].items()}, flush=True)"
  done
done
unset VCAP_LIB
