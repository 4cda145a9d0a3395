#!/bin/bash
# usage (GPU box): tools/gpu_tests.sh <outdir> [pytest selectors...]
out=${1:-gpurun_out/tests}; shift
mkdir -p $out
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -v -rA --timeout 170 --timeout-method thread -s > $out/pytest.log 2>&1
rc=$?
tail -40 $out/pytest.log
exit $rc
