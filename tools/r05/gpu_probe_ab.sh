#!/bin/bash
# Probe A/B: the trio's launch timings (1,000- and 20-step) under engine environment overrides.
#     tools/r05/gpu_probe_ab.sh TAG "65536 8192" "jt1:COG_TRIO_JT=1" "jt0:COG_TRIO_JT=0"
set -o pipefail
TAG=$1; SHAPES=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "$@"; do
    lab=${v%%:*}; envs=${v#*:}
    echo "== $lab rep $rep"
    env $envs timeout -k 10 120 tools/r05/bin/duoprobe trio $SHAPES > "$OUT/$lab.$rep.txt" 2>&1 || exit 1
    cat "$OUT/$lab.$rep.txt"
  done
done
