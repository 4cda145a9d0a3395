# rocprofv3 kernel trace + stats of the bench command (default: the driver's `--steps 20 --warmup 5`;
# the bench line's own live probe and the trace come from the same process) and its per-(kernel,
# grid) split (tools/kernel_trace_summary.py).  usage (GPU box): tools/prof_default.sh <outdir> [bench args]
set -e
out=${1:-gpurun_out/prof_default}; shift || true
args=${@:---steps 20 --warmup 5}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/trace -o run -- python3 $root/bench.py $args > $root/$out/bench.json 2> $root/$out/bench.err
f=$(find $root/$out/trace -name "run_kernel_trace.csv" | head -1)
python3 $root/tools/kernel_trace_summary.py $f > $root/$out/kernel_split.txt
s=$(find $root/$out/trace -name "run_kernel_stats.csv" | head -1)
cp $s $root/$out/kernel_stats.csv
echo done
