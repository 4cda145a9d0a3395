#!/bin/bash
# Validation of HEAD on one GPU box: the full GPU suite, smoke, the driver's bench command, its
# rocprofv3 kernel trace (fc1 mean vs the line's live probe) and the PMC passes (separate runs).
# Each step under its own limit; stops at the first step that ends in anything but pass / test failure.
# usage: tools/validate.sh <outdir> [nopmc]
out=${1:-gpurun_out/validate}
mkdir -p $out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -4 $out/gpu_tests.txt; ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $out/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/prof_default.sh $out/prof > $out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - $out <<'PY'
import json, sys, glob
out = sys.argv[1]
d = json.loads(open(f"{out}/prof/bench.json").read().strip().splitlines()[-1])
probe = d["roofline"]["avg_launch_ms"] * 1e3
rows = [l for l in open(f"{out}/prof/kernel_split.txt") if "gemm256_kernel<unsigned short, unsigned short, 1>" in l and "2364x1x1" in l]
mean = float(rows[0].split()[2]) if rows else float("nan")
print(f"fc1 16-video launches: probe {probe:.1f} us (bench line under rocprof), rocprof mean {mean:.1f} us, "
      f"ratio {mean / probe:.3f}")
PY
[ "$2" = nopmc ] && exit 0
bash tools/pmc.sh $out/pmc bench.py --serial --batch 16 --steps 2 --warmup 1 --host-e2e 0 --cpu-baseline-s 0 \
  --no-parity --no-decode-alone --strict-steps 0 --token-exact-steps 0 > $out/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_report.py $out/pmc 72 $out/pmc.json 50432 && echo "pmc report ok"
