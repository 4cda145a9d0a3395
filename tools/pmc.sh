#!/bin/bash
# usage (on the GPU box): tools/pmc.sh <outdir> <python script + args...>
# Three separate counter passes (never combined with sys/runtime traces): SQ utilisation and
# stall buckets, FETCH_SIZE, WRITE_SIZE (TCC slots cannot hold both).  Each pass: kernel trace +
# counters in CSV under <outdir>/<pass>/.
set -e
out=$1; shift
mkdir -p "$out"
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
pass() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$root/$out/$name" -o run -- python3 "${CMD[@]}" \
    > "$root/$out/$name.log" 2>&1
}
CMD=("$@")
CMD[0]="$root/${CMD[0]}"
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
echo "pmc passes done: $out"
