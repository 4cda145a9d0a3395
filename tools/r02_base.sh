set -e
mkdir -p gpurun_out/r02a
timeout -k 10 120 python tools/decode_step_time.py > gpurun_out/r02a/step.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02a/prof_dec -o run -- python3 $GRAFT_REPO_ROOT/tools/decode_step_time.py > $GRAFT_REPO_ROOT/gpurun_out/r02a/prof_dec.log 2>&1
echo ok
