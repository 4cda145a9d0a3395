#!/bin/bash
# usage (GPU box): tools/round_measure.sh <outdir>
# headline bench (configs[1], bf16) + its rocprofv3 kernel stats; configs[4]-shaped fp8 run (16 videos
# per GPU) + its kernel stats.  Every GPU step under its own time limit; stops at the first failure.
set -e
out=${1:-gpurun_out/measure}
mkdir -p $out
root=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python bench.py > $out/bench_bf16.json 2> $out/bench_bf16.err
timeout -k 10 300 python bench.py --precision fp8 --batch 16 --cpu-baseline-s 0 > $out/bench_fp8_b16.json 2> $out/bench_fp8_b16.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/prof_bf16 -o run -- python3 $root/bench.py --steps 5 --warmup 2 --cpu-baseline-s 0 > $root/$out/prof_bf16.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/prof_fp8 -o run -- python3 $root/bench.py --steps 5 --warmup 2 --cpu-baseline-s 0 --precision fp8 --batch 16 > $root/$out/prof_fp8.log 2>&1
echo done
