#!/bin/bash
# vcap_beam_params.max_blocks (ABI v14): beam tests, then the configs[3] lines with the pipeline's cap
# now reaching the beam searches.
out=${1:-gpurun_out/r5bcc}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_search.py tests/test_gpu_large.py tests/test_gpu_decode_tiles.py > $root/$out/tests.txt 2>&1 || { tail -30 $root/$out/tests.txt; exit 1; }
tail -2 $root/$out/tests.txt
C3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 4"
timeout -k 10 500 python -u bench.py $C3 > $root/$out/c3_bf16.json 2> $root/$out/c3_bf16.err || exit $?
timeout -k 10 500 python -u bench.py $C3 --dec-precision fp32 > $root/$out/c3_mixed.json 2> $root/$out/c3_mixed.err || exit $?
for f in c3_bf16 c3_mixed; do python3 -c "
import json
d=json.loads(open('$root/$out/$f.json').read().strip().splitlines()[-1])
p=d.get('parity') or {}
print('$f', round(d['value'],1), 'p50', round(d['p50_latency_ms'],1), {k: round(v,1) for k,v in d['stage_ms_p50'].items()}, 'cap', d['config']['decode_block_cap'], 'strict', round(d['strict_batch']['value'],1), 'step', round(d['decode_roofline']['step_us'],1), {k: p.get(k) for k in ('hypotheses_identical','max_score_deficit')})"; done
