#!/bin/bash
# bf16 gemv8 check: GPT-2-medium mlp c_proj (K = 4096) on the 8-wave GEMV - beam / decode tests, the
# configs[3] bf16 step; then GPT-2 small's K = 3072 on it (libvcap_g8s.so, -DVCAP_AB_GEMV8_SMALL)
# against the 4-wave kernel, greedy step alone at B = 8 and 16 rows capped at 96, interleaved.
# Both measured even and were removed (profiles/r05_beam_step_rework.txt); the variant flag no longer
# exists, so the second half now times the same library twice.
out=${1:-gpurun_out/r5g8}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_large.py tests/test_gpu_decode_tiles.py tests/test_gpu_search.py > $root/$out/tests.txt 2>&1 || { tail -30 $root/$out/tests.txt; exit 1; }
tail -2 $root/$out/tests.txt
for B in 8 4; do
  B=$B BEAMS=4 GPT2=gpt2-medium PREC=bf16 timeout -k 10 200 python3 tools/decode_step_time.py 2>&1 | grep step | tee -a $root/$out/steps.txt || exit 1
done
for rep in 1 2; do
  for lib in base g8s; do
    if [ $lib = base ]; then L=""; else L=$root/video-caption-algorithm_amd/vcap/_lib/libvcap_g8s.so; fi
    for cfg in "8 0" "16 96"; do
      set -- $cfg
      if [ -n "$L" ]; then
        VCAP_LIB=$L B=$1 CAP=$2 timeout -k 10 200 python3 tools/decode_step_time.py 2>&1 | grep step | sed "s/^/$lib /" | tee -a $root/$out/small.txt || exit 1
      else
        B=$1 CAP=$2 timeout -k 10 200 python3 tools/decode_step_time.py 2>&1 | grep step | sed "s/^/$lib /" | tee -a $root/$out/small.txt || exit 1
      fi
    done
  done
done
echo done
