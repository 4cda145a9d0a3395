#!/bin/bash
# usage: tools_prof.sh <outdir> <bench args...>   (run on the GPU box)
out=$1; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python bench.py "$@" > $out/bench.log 2>&1
