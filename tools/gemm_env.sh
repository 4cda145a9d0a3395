# ViT GEMM shapes (tools/gemm_bench.py [M]) under several environment settings, interleaved, same box
set -e
M=${M:-25216}
for rep in 1 2; do
  for e in "$@"; do
    echo "== $e"
    env $e timeout -k 10 180 python tools/gemm_bench.py $M 2>&1 | grep -v amdgpu | sed 's/tile128.*tile256/t256/'
  done
done
