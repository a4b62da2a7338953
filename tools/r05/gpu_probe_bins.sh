#!/bin/bash
# Probe A/B between probe binaries built from different engine sources (tools/r05/bin/<name>).
#     tools/r05/gpu_probe_bins.sh TAG "65536 8192" duoprobe_old duoprobe
set -o pipefail
TAG=$1; SHAPES=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for b in "$@"; do
    echo "== $b rep $rep"
    timeout -k 10 120 tools/r05/bin/$b trio $SHAPES > "$OUT/$b.$rep.txt" 2>&1 || exit 1
    cat "$OUT/$b.$rep.txt"
  done
done
