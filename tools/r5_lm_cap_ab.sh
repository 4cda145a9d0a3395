#!/bin/bash
# Greedy lm_head stream kernel grid capped at the decode cap (>= the 99 workgroups a GPT-2 vocabulary needs
# at <= 32 tiles each; libvcap_lmcap.so, -DVCAP_AB_LM_CAP) against one workgroup per CU: configs[1]
# bf16 and the bf16 / fp32-decoder split, ABAB, quick legs off, 40 timed batches. Measured +0.5 %
# (profiles/r05_lm_cap_ab.txt) and removed: the variant flag no longer exists.
out=${1:-gpurun_out/r5lmcap}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $out
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0 --steps 40"
for rep in 1 2; do
  for lib in base lmcap; do
    for P in bf16 fp32; do
      tag="${lib}_${P}_$rep"
      if [ $lib = base ]; then
        timeout -k 10 300 python -u bench.py $quick --dec-precision $P > $out/$tag.json 2> $out/$tag.err || exit $?
      else
        VCAP_LIB=$root/video-caption-algorithm_amd/vcap/_lib/libvcap_lmcap.so timeout -k 10 300 python -u bench.py $quick --dec-precision $P > $out/$tag.json 2> $out/$tag.err || exit $?
      fi
      python3 -c "
import json
d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1])
print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],2), {k: round(v,2) for k,v in d['stage_ms_p50'].items()})" | tee -a $out/summary.txt
    done
  done
done
