set -o pipefail
bash tools/ab.sh gpurun_out/r6b_te bench "|" "|--dec-precision fp32" "|--dec-precision fp32 --reserve-cus 48" "|--dec-precision fp32 --reserve-cus 64" "|--dec-precision fp32 --dec-group 4" "|--dec-precision fp32 --decode-blocks 128" > gpurun_out/r6b_te/summary.txt 2>&1
rc=$?; cat gpurun_out/r6b_te/summary.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --precision fp32 --steps 24 --warmup 3 > gpurun_out/r6b_c3_fp32.json 2> gpurun_out/r6b_c3_fp32.err
rc=$?; echo "c3 fp32 rc=$rc"; tail -c 1500 gpurun_out/r6b_c3_fp32.json; exit $rc
