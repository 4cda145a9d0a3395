#!/bin/bash
# ViT-L/14 fused QKV + attention (vcap_vit_qkv_attention_l_kernel): bit-identity tests, the kernel
# against the unfused pair at the configs[3] shape (8 videos x 32 frames, 257 tokens, 16 heads) and
# at ViT-B/16's, then the configs[3] bf16 line.
out=${1:-gpurun_out/r5l14}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_qkv_attention.py > $root/$out/tests.txt 2>&1 || { tail -40 $root/$out/tests.txt; exit 1; }
tail -3 $root/$out/tests.txt
BT=256 NT=257 H=16 timeout -k 10 200 python3 tools/qkv_attn_bench.py 2>&1 | grep -v amdgpu.ids | tee $root/$out/ab.txt || exit 1
BT=256 timeout -k 10 200 python3 tools/qkv_attn_bench.py 2>&1 | grep -v amdgpu.ids | tee -a $root/$out/ab.txt || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_large.py > $root/$out/large.txt 2>&1 || { tail -30 $root/$out/large.txt; exit 1; }
tail -2 $root/$out/large.txt
C3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 4"
timeout -k 10 500 python -u bench.py $C3 > $root/$out/c3_bf16.json 2> $root/$out/c3_bf16.err || exit $?
python3 -c "
import json
d=json.loads(open('$root/$out/c3_bf16.json').read().strip().splitlines()[-1])
print('c3_bf16', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), d['stage_ms_p50'], d['attention']['kernel'], round(d['attention']['avg_launch_ms']*1e3,1), 'us')"
