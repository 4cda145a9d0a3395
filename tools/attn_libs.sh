# ViT attention alone (tools/attn_bench.py) on several library builds, interleaved, same box
set -e
L=video-caption-algorithm_amd/vcap/_lib
for rep in 1 2; do
  for lib in "$@"; do
    echo -n "$lib: "
    VCAP_LIB=$L/$lib.so BT=${BT:-128} timeout -k 10 120 python tools/attn_bench.py
  done
done
