#!/bin/bash
# Marginal cost of each decode kernel in the dependent chain: step time with that kernel launched
# twice per layer (VCAP_DECODE_DUP) minus the baseline step time (tools/decode_step_time.py).
for m in 0 1 2 4 8 16; do
  VCAP_DECODE_DUP=$m timeout -k 10 120 python tools/decode_step_time.py 2>/dev/null | sed "s/^/dup=$m /" || exit 1
done
