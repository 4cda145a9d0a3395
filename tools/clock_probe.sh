#!/bin/bash
# Sample the GPU's power and clocks (rocm-smi, read-only) while (1) the encode runs alone in a loop
# and (2) the pipelined bench runs: is the encode's ~10 % slowdown beside the decodes a clock drop?
out=${1:-gpurun_out/clk}; mkdir -p $out
sample() { while true; do echo "t $(date +%s.%N)"; rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Power|sclk|mclk|fclk"; sleep 0.2; done; }
sample > $out/smi_encode.log & S=$!
ITERS=500 timeout -k 10 180 python tools/encode_split.py > $out/encode.log 2>&1; rc=$?
kill $S; [ $rc -eq 0 ] || exit $rc
sample > $out/smi_bench.log & S=$!
timeout -k 10 180 python bench.py --steps 800 --warmup 4 --cpu-baseline-s 0 --host-e2e 0 --no-parity --no-decode-alone > $out/bench.json 2> $out/bench.err; rc=$?
kill $S; exit $rc
