#!/bin/bash
# Round-4 milestone validation on one GPU box: the full GPU suite, smoke, the driver's bench command
# and the default bench; each step under its own time limit, stopping at the first step that ends in
# anything but pass / test failure.  usage: tools/r4_validate.sh <outdir> [pmc]
out=${1:-gpurun_out/validate}
mkdir -p $out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -8 $out/gpu_tests.txt; ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $out/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $out/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err
rc=$?; echo "default bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ "$2" = pmc ]; then bash tools/r4_pmc.sh $out/pmc > $out/pmc.log 2>&1; rc=$?; echo "pmc rc=$rc"; tail -12 $out/pmc.log; fi
exit $rc
