# ViT GEMM shapes (tools/gemm_bench.py) on several library builds, interleaved, same box
set -e
L=video-caption-algorithm_amd/vcap/_lib
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib"
    VCAP_LIB=$L/$lib.so timeout -k 10 180 python tools/gemm_bench.py 2>&1 | grep -v amdgpu
  done
done
