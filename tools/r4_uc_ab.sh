#!/bin/bash
# Decoder weights in uncached device memory (bench.py --uc-decode-weights) vs default, interleaved;
# the decode step alone and parity legs on.  usage: tools/r4_uc_ab.sh OUTDIR
out=${1:-gpurun_out/uc}
mkdir -p "$out"
quick="--host-e2e 0 --cpu-baseline-s 0 --strict-steps 0"
for i in 1 2; do
  for f in "" "--uc-decode-weights"; do
    tag="uc$([ -n "$f" ] && echo 1 || echo 0)_$i"
    timeout -k 10 300 python -u bench.py $quick $f > "$out/$tag.json" 2> "$out/$tag.err" || exit $?
    python3 -c "import json; d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1), 'dec step', round(d['decode_roofline']['step_us'],1), 'fc1', round(d['roofline']['avg_launch_ms']*1e3,1), 'parity', d['parity']['captions_identical'], {k: round(v,2) for k, v in d['stage_ms_p50'].items()})" | tee -a "$out/summary.txt"
  done
done
