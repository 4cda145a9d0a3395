#!/bin/bash
# Round-4 extra bench lines (one GPU): the reference's batch-size sweep and the two fp8 lines
# (all four ViT GEMMs in MXFP8, and QKV + attn-proj only with the MLP in bf16).
# usage: bash tools/r4_lines.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/lines}
mkdir -p "$out"
timeout -k 10 420 python -u bench.py --batch-sizes 1,2,4,8,12,16 --steps 30 > "$out/sweep.json" 2> "$out/sweep.err" &&
timeout -k 10 240 python -u bench.py --precision fp8 --batch 16 --steps 30 > "$out/fp8_all4.json" 2> "$out/fp8_all4.err" &&
timeout -k 10 240 python -u bench.py --precision fp8 --batch 16 --steps 30 --mx-gemms qkv,proj > "$out/fp8_qkv_proj.json" 2> "$out/fp8_qkv_proj.err"
rc=$?
echo "lines rc=$rc"
exit $rc
