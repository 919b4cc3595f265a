#!/bin/bash
# Same-box ResNet-50 A/B between tree copies: bench/ab_r50.sh OUT DIR1 DIR2 ...  ("." = the current tree), 2 rounds
out=$1
shift
: > "$out"
for rep in 1 2; do
  for d in "$@"; do
    echo "== $d rep=$rep" >> "$out"
    (cd "$d" && timeout -k 10 200 python bench/resnet50.py --steps 30 --warmup 5 2>/dev/null | grep metric) >> "$out" || exit 1
  done
done
