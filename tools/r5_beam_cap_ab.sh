#!/bin/bash
# configs[3]: the beam decode's GEMV grids and beam lm_head capped at 96 workgroups (libvcap_bcap.so,
# -DVCAP_AB_BEAM_CAP=96) against uncapped beam decodes, bf16 and fp32 decoder, ABAB, quick legs off.
out=${1:-gpurun_out/r5bcap}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $out
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
C3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 4"
for rep in 1 2; do
  for lib in base bcap; do
    for P in bf16 fp32; do
      tag="${lib}_${P}_$rep"
      if [ $lib = base ]; then
        timeout -k 10 400 python -u bench.py $C3 $quick --dec-precision $P > $out/$tag.json 2> $out/$tag.err || exit $?
      else
        VCAP_LIB=$root/video-caption-algorithm_amd/vcap/_lib/libvcap_bcap.so timeout -k 10 400 python -u bench.py $C3 $quick --dec-precision $P > $out/$tag.json 2> $out/$tag.err || exit $?
      fi
      python3 -c "
import json
d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1])
print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,1) for k,v in d['stage_ms_p50'].items()})" | tee -a $out/summary.txt
    done
  done
done
