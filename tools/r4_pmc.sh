#!/bin/bash
# Round-4 PMC pass of HEAD on the configs[1] encode shape (16-video encodes, 50432 ViT rows per GEMM
# launch, as the default bench's enc_group 2): three separate counter passes (tools/pmc.sh), then
# the per-kernel report with attn-proj and fc2 split.  usage (GPU box): tools/r4_pmc.sh <outdir>
out=${1:-gpurun_out/pmc_r4}
bash tools/pmc.sh $out bench.py --serial --batch 16 --steps 2 --warmup 1 --host-e2e 0 --cpu-baseline-s 0 \
  --no-parity --no-decode-alone --strict-steps 0 || exit $?
python3 tools/pmc_report.py $out 72 $out/pmc.json 50432
