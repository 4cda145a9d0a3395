#!/bin/bash
# A/B of the 256x256 GEMM's column-group tile order for fc1 (VCAP_GEMM_COLGROUP=w) on one box:
# the GEMM alone (tools/gemm_bench.py at 50432 rows), the pipelined bench interleaved (quick legs
# off), then one PMC pass with the grouped order.  usage: tools/r4_colgroup_ab.sh OUTDIR [w]
out=${1:-gpurun_out/cg}
w=${2:-6}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for cg in 0 $w; do
  VCAP_GEMM_COLGROUP=$cg timeout -k 10 120 python -u tools/gemm_bench.py 50432 > "$out/gemm_cg$cg.txt" 2>&1 || exit $?
done
for i in 1 2; do
  for cg in 0 $w; do
    VCAP_GEMM_COLGROUP=$cg timeout -k 10 300 python -u bench.py $quick > "$out/bench_cg${cg}_$i.json" 2> "$out/bench_cg${cg}_$i.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open('$out/bench_cg${cg}_$i.json').read().strip().splitlines()[-1]); print('cg=$cg run $i', round(d['value'],1), 'fc1 us', round(d['roofline']['avg_launch_ms']*1e3,1))"
  done
done
VCAP_GEMM_COLGROUP=$w bash tools/r4_pmc.sh "$out/pmc" > "$out/pmc.log" 2>&1
rc=$?
echo "pmc rc=$rc"
exit $rc
