#!/bin/bash
# A/B of the in-step gradient reduction (DCA_PKS_RED_IN_STEP) on one box: 3 alternating runs each, 300 steps.
set -o pipefail
out=${1:-gpurun_out/ab_red.log}
: > "$out"
for rep in 1 2 3; do
  for v in 1 0; do
    echo "== red_in_step=$v rep=$rep" >> "$out"
    DCA_PKS_RED_IN_STEP=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 >> "$out" 2>/dev/null || exit 1
  done
done
