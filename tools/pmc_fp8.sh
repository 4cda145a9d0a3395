#!/bin/bash
# rocprofv3 PMC passes (tools/pmc.sh) of the configs[4]-shaped MXFP8 encode at 16 videos (serial, so
# each launch is counted alone) -> <outdir>/pmc_fp8.json.  usage (GPU box): tools/pmc_fp8.sh <outdir>
out=${1:-gpurun_out/pmc_fp8}
bash tools/pmc.sh $out/pmc bench.py --precision fp8 --serial --batch 16 --steps 2 --warmup 1 --host-e2e 0 \
  --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0 --token-exact-steps 0 > $out.log 2>&1 || exit $?
python3 tools/pmc_report.py $out/pmc 72 $out/pmc_fp8.json 50432
