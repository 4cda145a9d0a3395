#!/bin/bash
# One GPU-box session: selected GPU tests, then (optionally) the full GPU suite and the default bench.
# usage: tools/gpu_round.sh <outdir> "<pytest selectors>" [full] [bench] [bench args...]
# Stops at the first step that ends in anything but pass / test failure (timeout, abort, segfault).
out=${1:-gpurun_out/r}; sel=$2; shift 2
mkdir -p $out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
rc=0
if [ -n "$sel" ]; then
  timeout -k 10 900 python -u -m pytest $sel -m gpu -v -rA --timeout 300 --timeout-method thread -s > $out/sel.log 2>&1
  rc=$?; echo "selected tests rc=$rc"; tail -25 $out/sel.log
  ok $rc || exit $rc
fi
if [ "$1" = full ]; then
  shift
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/full.log 2>&1
  rc=$?; echo "full suite rc=$rc"; tail -15 $out/full.log
  ok $rc || exit $rc
fi
if [ "$1" = bench ]; then
  shift
  timeout -k 10 400 python -u bench.py "$@" > $out/bench.json 2> $out/bench.err
  rc=$?; echo "bench rc=$rc"; tail -c 3000 $out/bench.json; tail -5 $out/bench.err
fi
exit $rc
