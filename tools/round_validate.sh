#!/bin/bash
# End-of-milestone validation on one GPU box: the full GPU suite, the driver's bench command, the
# configs[4]-shaped fp8 line and the configs[3] line, each under its own time limit; stops at the
# first step that ends in anything but pass / test failure.  usage: tools/round_validate.sh <outdir>
out=${1:-gpurun_out/validate}
mkdir -p $out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -4 $out/gpu_tests.txt; ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $out/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $out/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err
rc=$?; echo "default bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --precision fp8 --batch 16 --steps 20 --warmup 5 > $out/bench_fp8.json 2> $out/bench_fp8.err
rc=$?; echo "fp8 bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 3 > $out/bench_c3.json 2> $out/bench_c3.err
rc=$?; echo "c3 bench rc=$rc"; exit $rc
