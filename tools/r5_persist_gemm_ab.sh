#!/bin/bash
# Persistent 256x256 GEMM grid (gemm policy | 4) vs one tile per workgroup: bit-identity, then the
# driver-shaped bench interleaved on one box (encode stage, fc1 probe, captions/s).
out=${1:-gpurun_out/r5pg}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -q -k "bitwise_equal" --timeout 200 --timeout-method thread > $out/tests.txt 2>&1; rc=$?; tail -2 $out/tests.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for P in 0 4; do
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --gemm-policy $P --cpu-baseline-s 0 --no-parity --no-decode-alone --host-e2e 0 --strict-steps 0 > $out/b_${P}_$i.json 2> $out/b_${P}_$i.err || exit $?
  python3 -c "
import json; d=json.loads(open('$out/b_${P}_$i.json').read().strip().splitlines()[-1])
print('policy $P run $i', round(d['value'],1), 'p50', round(d['p50_latency_ms'],2), d['stage_ms_p50'], 'fc1', round(d['roofline']['avg_launch_ms']*1e3,1), 'attn', round(d['attention']['avg_launch_ms']*1e3,1))"
done; done
