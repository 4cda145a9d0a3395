#!/bin/bash
# usage: tools/kernel_resources.sh <file.hip> -> per-kernel VGPR / AGPR / spill summary (gfx950)
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/gpurun_out/scratch; mkdir -p $out
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I$root/video-caption-algorithm_amd/csrc -I$root/include \
  -c "$1" -Rpass-analysis=kernel-resource-usage -o $out/res.o 2>&1 | python3 -c "
import sys, re
cur = None
for line in sys.stdin:
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = m.group(1); print(); print(cur[:70], end=' ')
    m = re.search(r'(VGPRs|AGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)', line)
    if m and cur:
        print(m.group(1).split()[0] + ('S' if 'Spill' in m.group(1) else '') + '=' + m.group(2), end=' ')
print()
"
