#!/bin/bash
# One A/B runner for every "same box, interleaved" comparison (replaces r01-r02's per-experiment
# scripts).  usage (GPU box):
#   tools/ab.sh <outdir> <runner> <spec> [<spec> ...]
# runner: bench   python bench.py (quick leg: no CPU baseline / host e2e / parity / decode-alone)
#         gemm    tools/gemm_bench.py        (ViT GEMM shapes alone)
#         attn    tools/attn_bench.py        (ViT attention alone; BT from the environment)
#         decode  tools/decode_step_time.py  (decode step alone; B from the environment)
# spec:   "<ENV=V ...>|<args>"  - environment (e.g. VCAP_LIB=<path to a variant build>, made with
#         VCAP_LIB_NAME / VCAP_EXTRA_FLAGS through vcap.build or tools/build_ref_lib.sh) and
#         runner arguments; either side may be empty.  Every spec runs twice, interleaved.
out=$1; runner=$2; shift 2
mkdir -p $out
case $runner in
  bench)  cmd="python bench.py --cpu-baseline-s 0 --host-e2e 0 --no-parity --no-decode-alone --strict-steps 0 --token-exact-steps 0" ;;
  gemm)   cmd="python tools/gemm_bench.py" ;;
  attn)   cmd="python tools/attn_bench.py" ;;
  decode) cmd="python tools/decode_step_time.py" ;;
  *) echo "unknown runner $runner"; exit 2 ;;
esac
i=0
for rep in 1 2; do
  for spec in "$@"; do
    i=$((i+1))
    e=${spec%%|*}; a=${spec#*|}
    [ "$spec" = "${spec#*|}" ] && a=""
    env $e timeout -k 10 300 $cmd $a > $out/r$i.out 2> $out/r$i.err || { echo "run $i ($spec) failed"; tail -5 $out/r$i.err; exit 1; }
    if [ $runner = bench ]; then
      python3 -c "
import json;d=json.loads(open('$out/r$i.out').read().strip().splitlines()[-1])
print('$spec |', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'p50', round(d['p50_latency_ms'],1), {k: round(v,2) for k,v in d['stage_ms_p50'].items()})"
    else
      echo "$spec | $(grep -v amdgpu $out/r$i.out | tr '\n' ' ')"
    fi
  done
done
