#!/bin/bash
# Round 5: the fused c_attn + attention decode - its bit-identity tests first, the decode step alone
# split vs fused, then the full GPU suite and the driver's bench command.  Each step under its own
# limit; stops at the first step that ends in anything but pass / test failure.
# usage: tools/r5_decode_check.sh <outdir>
out=${1:-gpurun_out/r5}
mkdir -p $out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_fused.py -x -q -rf --timeout 120 --timeout-method thread > $out/fused_tests.txt 2>&1
rc=$?; echo "fused tests rc=$rc"; tail -5 $out/fused_tests.txt; ok $rc || exit $rc
for B in 8 16; do for CAP in 0 96; do for SPLIT in 1 0 1 0; do
  B=$B CAP=$CAP SPLIT=$SPLIT timeout -k 10 120 python -u tools/decode_step_time.py >> $out/step_time.txt 2>&1 || exit $?
done; done; done
cat $out/step_time.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -8 $out/gpu_tests.txt; ok $rc || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $out/bench.json; exit $rc
