#!/bin/bash
# fp32 decoder changes: parity tests (fp32 token-exact vs goldens, logits 1e-3), decode step timing, mixed bench line.
out=${1:-gpurun_out/r5f}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_search.py tests/test_gpu_large.py tests/test_gpu_decode_tiles.py tests/test_gpu_surface.py -x -q --timeout 300 --timeout-method thread > $out/tests.txt 2>&1; rc=$?; tail -3 $out/tests.txt; [ $rc -eq 0 ] || exit $rc
for B in 8 16; do for CAP in 0 96; do
  B=$B CAP=$CAP PREC=fp32 timeout -k 10 120 python -u tools/decode_step_time.py 2>/dev/null | grep step >> $out/step.txt || exit 1
done; done
cat $out/step.txt
timeout -k 10 400 python -u bench.py --dec-precision fp32 --steps 20 --warmup 5 > $out/mixed.json 2> $out/mixed.err || exit $?
python3 -c "
import json; d=json.loads(open('$out/mixed.json').read().strip().splitlines()[-1])
print('mixed', round(d['value'],1), 'p50', round(d['p50_latency_ms'],2), d['stage_ms_p50'], 'step', round(d['decode_roofline']['step_us'],1), 'oracle', d['oracle_parity']['captions_identical'], 'parity', d['parity']['captions_identical'])"
