#!/bin/bash
# usage (GPU box): tools/round_measure.sh <outdir>
# headline bench (configs[1], bf16) + its rocprofv3 kernel stats; configs[4]-shaped fp8 run (16 videos
# per GPU); configs[3] (L/14 + GPT-2-medium, 32 frames, beam 4) + its kernel stats.  Every GPU step
# under its own time limit; stops at the first failure.
set -e
out=${1:-gpurun_out/measure}
mkdir -p $out
root=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python bench.py > $out/bench_bf16.json 2> $out/bench_bf16.err
timeout -k 10 300 python bench.py --precision fp8 --batch 16 --cpu-baseline-s 0 > $out/bench_fp8_b16.json 2> $out/bench_fp8_b16.err
timeout -k 10 400 python bench.py --vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 \
  --max-new 40 --steps 10 --warmup 2 --cpu-baseline-s 15 > $out/bench_c3.json 2> $out/bench_c3.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/prof_bf16 -o run -- python3 $root/bench.py --steps 6 --warmup 2 --cpu-baseline-s 0 --no-parity --host-e2e 0 > $root/$out/prof_bf16.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/prof_c3 -o run -- python3 $root/bench.py --vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 4 --warmup 2 --cpu-baseline-s 0 --no-parity --host-e2e 0 > $root/$out/prof_c3.log 2>&1
echo done
