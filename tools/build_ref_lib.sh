#!/bin/bash
# usage: tools/build_ref_lib.sh <git-rev> <out.so>   build libvcap_hip.so from the sources of <git-rev>
# (scratch under gpurun_out/, which never ships) for same-process / same-box A/B runs
set -e
rev=$1; out=$2
root=$(cd "$(dirname "$0")/.." && pwd)
d=$root/gpurun_out/refbuild/$rev; rm -rf $d; mkdir -p $d/csrc $d/include $d/obj
for f in $(git -C $root ls-tree --name-only $rev video-caption-algorithm_amd/csrc/); do
  git -C $root show $rev:$f > $d/csrc/$(basename $f); done
git -C $root show $rev:include/vcap.h > $d/include/vcap.h
mkdir -p $d/../include && cp $d/include/vcap.h $d/../include/vcap.h   # runtime.hip includes ../../include/vcap.h
for f in $d/csrc/*.hip; do
  extra=""; [ "$(basename $f)" = vit_attention.hip ] && extra="-fno-honor-nans"   # as vcap/build.py FILE_FLAGS
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result $extra \
    -I$d/csrc -I$d/include -c $f -o $d/obj/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $d/obj/*.o
echo "$out <- $rev"
