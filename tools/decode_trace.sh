# rocprofv3 kernel trace of the decode alone (tools/decode_step_time.py) and its per-kernel split:
# which kernel of the ~62-launch token step takes how long.  usage (GPU box): tools/decode_trace.sh <outdir> [B]
set -e
out=${1:-gpurun_out/decode_trace}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
cd /tmp && export TMPDIR=/tmp
B=${2:-8} timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $root/$out/trace -o run -- python3 $root/tools/decode_step_time.py > $root/$out/run.log 2>&1
f=$(find $root/$out/trace -name "run_kernel_trace.csv" | head -1)
python3 $root/tools/kernel_trace_summary.py $f > $root/$out/kernel_split.txt
echo done
