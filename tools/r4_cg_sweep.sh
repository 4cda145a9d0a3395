#!/bin/bash
# fc1 column-group width under the default schedule (VCAP_GEMM_COLGROUP 0 = row-major, 3, 4, 6 =
# the default), then configs[3] (ViT-L/14 fc1: 16 tiles of 512 KB, default group 4) row-major vs
# default.  Quick legs off.  usage: tools/r4_cg_sweep.sh OUTDIR
out=${1:-gpurun_out/cgw}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for w in 0 3 4 6 0 6; do
  VCAP_GEMM_COLGROUP=$w timeout -k 10 300 python -u bench.py $quick > "$out/b_$w.json" 2> "$out/b_$w.err" || exit $?
  python3 -c "import json; d=json.loads(open('$out/b_$w.json').read().strip().splitlines()[-1]); print('configs[1] colgroup=$w', round(d['value'],1), 'fc1 us', round(d['roofline']['avg_launch_ms']*1e3,1))" | tee -a "$out/summary.txt"
done
c3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 16 --warmup 2"
for w in 0 4 0 4; do
  VCAP_GEMM_COLGROUP=$w timeout -k 10 400 python -u bench.py $quick $c3 > "$out/c3_$w.json" 2> "$out/c3_$w.err" || exit $?
  python3 -c "import json; d=json.loads(open('$out/c3_$w.json').read().strip().splitlines()[-1]); print('configs[3] colgroup=$w', round(d['value'],2), 'fc1 us', round(d['roofline']['avg_launch_ms']*1e3,1))" | tee -a "$out/summary.txt"
done
