#!/bin/bash
# Same-box A/B matrix: the round-3 tree (.r3base/) and the current tree under env knob settings; 300-step bench runs,
# interleaved.  Usage: bench/ab_matrix.sh OUT "label|ENV=.. ENV=.." ...   (label r3 = the round-3 tree; a label X
# with a directory .X = that scratch copy of the tree)
set -o pipefail
out=$1
shift
: > "$out"
for rep in 1 2; do
  for spec in "$@"; do
    label=${spec%%|*}
    envs=${spec#*|}
    echo "== $label rep=$rep" >> "$out"
    if [ "$label" = r3 ]; then
      (cd .r3base && timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-fp32) >> "$out" 2>/dev/null || exit 1
    elif [ -d ".$label" ]; then  # a scratch copy of the tree (gitignored) with one change reverted
      (cd ".$label" && env $envs timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-fp32) >> "$out" 2>/dev/null || exit 1
    else
      env $envs timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-fp32 >> "$out" 2>/dev/null || exit 1
    fi
  done
done
