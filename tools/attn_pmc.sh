# PMC passes over tools/attn_bench.py (shipped attention kernel): instruction mix and stall buckets
set -e
out=${1:-gpurun_out/attn_pmc}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $root/$out/avail.txt 2>&1 || true
p() { n=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $root/$out/$n -o run -- python3 $root/tools/attn_bench.py > $root/$out/$n.log 2>&1; }
p a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
p b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
echo done
