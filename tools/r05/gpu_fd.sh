#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r05fd}; mkdir -p "$OUT"
for k in wave pipe duo; do
  for n in 65536 16384; do
    COG_ROLLOUT=$k timeout -k 10 120 python tools/r05/fd_kinds.py $n >> "$OUT/fd.txt" 2>&1 || exit 1
  done
done
cat "$OUT/fd.txt"
