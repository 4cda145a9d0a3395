#!/bin/bash
# usage (GPU box): tools/lanes_sweep.sh <outdir> ["lanes..."] ["reserve..."] [extra bench args]
# bench.py (B=8 bf16 overlapped) over decode lanes x encode CU reservation; one JSON line per run.
set -e
out=${1:-gpurun_out/lanes}; lanes=${2:-"1 2"}; res=${3:-"64 96 128"}; extra=${4:-}
mkdir -p $out
for l in $lanes; do for r in $res; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 4 --cpu-baseline-s 0 --dec-lanes $l --reserve-cus $r $extra \
    > $out/l${l}_r${r}.json 2> $out/l${l}_r${r}.err
  python - "$out/l${l}_r${r}.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d['value'], 1), round(d['ms_per_step'], 2), round(d['p50_latency_ms'], 2),
      {k: round(v, 2) for k, v in d['stage_ms_p50'].items()}, flush=True)
PY
done; done
