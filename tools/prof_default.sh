# rocprofv3 kernel trace + stats of the DEFAULT bench command (the bench line's own live probe and
# the trace come from the same process); usage (GPU box): tools/prof_default.sh <outdir>
set -e
out=${1:-gpurun_out/prof_default}
root=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $root/$out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/trace -o run -- python3 $root/bench.py > $root/$out/bench.json 2> $root/$out/bench.err
echo done
