# decode step alone (tools/decode_step_time.py, B rows) on several library builds, interleaved
set -e
L=video-caption-algorithm_amd/vcap/_lib
for rep in 1 2; do
  for lib in "$@"; do
    VCAP_LIB=$L/$lib.so B=${B:-8} timeout -k 10 120 python tools/decode_step_time.py
  done
done
