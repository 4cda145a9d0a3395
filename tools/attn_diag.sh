# ViT attention A/B: shipped vs pipelined kernel, each with compute or loads compiled out
# (libvcap_nocomp.so / libvcap_noload.so built with -DVCAP_DIAG_ATTN_NOCOMP / _NOLOAD)
set -e
L=video-caption-algorithm_amd/vcap/_lib
for lib in libvcap_hip libvcap_nocomp libvcap_noload; do
  for p in 0 1; do
    echo -n "$lib pipe=$p: "
    VCAP_LIB=$L/$lib.so VCAP_ATTN_PIPE=$p BT=${BT:-128} timeout -k 10 120 python tools/attn_bench.py
  done
done
