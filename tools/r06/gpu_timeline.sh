#!/bin/bash
# The trio's launch timeline and per-phase ticks at the driver's shape (20-step launches), the
# multi-block grid on and off, the plain probe's timings beside a probe built from the round-5
# engine (tools/r06/bin/duoprobe_r05, same box), and the dependent-chain costs (chainprobe).
#     tools/r06/gpu_timeline.sh TAG
set -o pipefail
TAG=${1:-r06t}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for mb in 1 0; do
    COG_TRIO_MB=$mb timeout -k 10 120 tools/r06/bin/duoprobe trio 65536 8192 >> "$OUT/probe_mb$mb.txt" 2>&1 || exit 1
  done
  if [ -x tools/r06/bin/duoprobe_r05 ]; then
    timeout -k 10 120 tools/r06/bin/duoprobe_r05 trio_r05 65536 8192 >> "$OUT/probe_r05.txt" 2>&1 || exit 1
  fi
done
for mb in 1 0; do
  COG_TRIO_MB=$mb PROBE_CHUNK=20 PROBE_JSON=1 timeout -k 10 120 tools/r06/bin/duoprobe_st trio 65536 > "$OUT/stamps20_mb$mb.txt" 2>&1 || exit 1
done
timeout -k 10 60 tools/r06/bin/chainprobe > "$OUT/chainprobe.txt" 2>&1
cat "$OUT"/probe_*.txt "$OUT/chainprobe.txt"
