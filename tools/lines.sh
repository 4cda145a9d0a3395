#!/bin/bash
# The configs[4]-shaped fp8 line and the configs[3] lines (bf16 and fp32 end to end, the latter
# token-exact against the CPU oracle), each under its own limit, on one GPU box.
# usage: tools/lines.sh <outdir>
out=${1:-gpurun_out/lines}
mkdir -p $out
timeout -k 10 600 python -u bench.py --precision fp8 --batch 16 --steps 20 --warmup 5 > $out/bench_fp8.json 2> $out/bench_fp8.err
rc=$?; echo "fp8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
C3="--vit vit_large_patch14_224 --gpt2 gpt2-medium --frames 32 --batch 4 --beams 4 --max-new 40 --steps 24 --warmup 3"
timeout -k 10 700 python -u bench.py $C3 > $out/bench_c3_bf16.json 2> $out/bench_c3_bf16.err
rc=$?; echo "c3 bf16 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py $C3 --precision fp32 > $out/bench_c3_fp32.json 2> $out/bench_c3_fp32.err
rc=$?; echo "c3 fp32 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - $out <<'PY'
import json, sys
out = sys.argv[1]
for n in ("bench_fp8", "bench_c3_bf16", "bench_c3_fp32"):
    d = json.loads(open(f"{out}/{n}.json").read().strip().splitlines()[-1])
    par, op = d.get("parity") or {}, d.get("oracle_parity") or {}
    print(n, round(d["value"], 1), "p50", round(d["p50_latency_ms"], 1), "fc1", round(d["roofline"]["avg_launch_ms"] * 1e3, 1),
          "us frac", round(d["roofline"]["frac"], 3), "parity", par.get("captions_identical", par.get("hypotheses_identical")),
          "oracle", op.get("captions_identical"))
PY
