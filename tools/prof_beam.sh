cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${PB_DIR:-r02pb} -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_beam_step.py > $GRAFT_REPO_ROOT/gpurun_out/${PB_DIR:-r02pb}.log 2>&1
