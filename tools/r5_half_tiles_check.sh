mkdir -p gpurun_out/r5e
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_tiles.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5e/tiles.txt 2>&1; rc=$?; tail -3 gpurun_out/r5e/tiles.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for B in 8 16; do for CAP in 0 96; do for P in bf16 fp32; do
  B=$B CAP=$CAP PREC=$P timeout -k 10 120 python -u tools/decode_step_time.py 2>/dev/null | grep step >> gpurun_out/r5e/step.txt || exit 1
done; done; done
cat gpurun_out/r5e/step.txt
