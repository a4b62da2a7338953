#!/bin/bash
# Probe A/B between the engine of the previous commit (duoprobe_old) and the working tree's.
#     tools/r05/gpu_probe_old.sh TAG "65536 8192"
set -o pipefail
TAG=$1; SHAPES=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2 3; do
  for b in duoprobe_old duoprobe; do
    echo "== $b rep $rep"
    timeout -k 10 120 tools/r05/bin/$b trio $SHAPES > "$OUT/$b.$rep.txt" 2>&1 || exit 1
    cat "$OUT/$b.$rep.txt"
  done
done
