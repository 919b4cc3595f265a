#!/bin/bash
# Same-box A/B against the round-3 tree (.r3base/, gitignored, built in-tree): alternating 300-step bench runs.
set -o pipefail
out=${1:-gpurun_out/ab_r3.log}
: > "$out"
for rep in 1 2 3; do
  echo "== r3 rep=$rep" >> "$out"
  (cd .r3base && timeout -k 10 120 python bench.py --steps 300 --warmup 30) >> "$out" 2>/dev/null || exit 1
  echo "== r4 rep=$rep" >> "$out"
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 >> "$out" 2>/dev/null || exit 1
done
