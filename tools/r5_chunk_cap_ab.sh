#!/bin/bash
# configs[3] fp32 decoder: the decode grid cap divided over the 16-row chunks of the f32 GEMVs
# (libvcap_ccap.so, -DVCAP_AB_CHUNK_CAP) against the cap per chunk, ABAB, quick legs off. Not adopted
# (profiles/r05_chunk_cap_ab.txt); the variant flag no longer exists.
out=${1:-gpurun_out/r5ccap}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $out
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
C3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 4"
for rep in 1 2; do
  for lib in base ccap; do
    tag="${lib}_fp32_$rep"
    if [ $lib = base ]; then
      timeout -k 10 400 python -u bench.py $C3 $quick --dec-precision fp32 > $out/$tag.json 2> $out/$tag.err || exit $?
    else
      VCAP_LIB=$root/video-caption-algorithm_amd/vcap/_lib/libvcap_ccap.so timeout -k 10 400 python -u bench.py $C3 $quick --dec-precision fp32 > $out/$tag.json 2> $out/$tag.err || exit $?
    fi
    python3 -c "
import json
d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1])
print('$tag', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,1) for k,v in d['stage_ms_p50'].items()})" | tee -a $out/summary.txt
  done
done
