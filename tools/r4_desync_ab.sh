#!/bin/bash
# ViT attention first-round desync A/B (VCAP_ATTN_DESYNC=0/1): alone at 8 and 16 videos (outputs
# compared bit for bit), then the pipelined bench interleaved.  usage: tools/r4_desync_ab.sh OUTDIR
out=${1:-gpurun_out/desync}
mkdir -p "$out"
for bt in 128 256; do
  for d in 0 1; do
    BT=$bt DUMP=$out/attn_${bt}_$d.pt VCAP_ATTN_DESYNC=$d timeout -k 10 60 python -u tools/attn_bench.py >> "$out/alone.txt" 2>&1 || exit $?
    echo "^ BT=$bt desync=$d" >> "$out/alone.txt"
  done
  python3 -c "import torch; a=torch.load('$out/attn_${bt}_0.pt'); b=torch.load('$out/attn_${bt}_1.pt'); print('BT=$bt bit-identical', torch.equal(a, b))" >> "$out/alone.txt" || exit $?
done
rm -f $out/*.pt
quick="--host-e2e 0 --cpu-baseline-s 0 --no-parity --no-decode-alone --strict-steps 0"
for i in 1 2; do
  for d in 0 1; do
    VCAP_ATTN_DESYNC=$d timeout -k 10 300 python -u bench.py $quick > "$out/bench_${d}_$i.json" 2> "$out/bench_${d}_$i.err" || exit $?
    python3 -c "import json; d=json.loads(open('$out/bench_${d}_$i.json').read().strip().splitlines()[-1]); a=d['attention']; print('desync=$d run $i', round(d['value'],1), 'attention us', round(a['avg_launch_ms']*1e3,1), {k: round(v,2) for k, v in d['stage_ms_p50'].items()})" | tee -a "$out/bench.txt"
  done
done
