#!/bin/bash
# PMC passes over tools/qkv_attn_bench.py (fused QKV + attention vs the unfused pair), one counter
# set per rocprofv3 run: SQ utilisation / stall buckets, L2 hit / miss, FETCH_SIZE.
# usage (GPU box): tools/qa_pmc.sh <outdir>
set -e
out=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$root/$out"
cd /tmp && export TMPDIR=/tmp
pass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$root/$out/$name" -o run -- \
    python3 "$root/tools/qkv_attn_bench.py" > "$root/$out/$name.log" 2>&1
}
export REPS=2
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
pass tcc TCC_HIT_sum TCC_MISS_sum
pass fetch FETCH_SIZE
echo "qa pmc done: $out"
