#!/bin/bash
# Diagnostic: trio launch timings (1,000- / 20-step, and 1 / 2 / 5-step launches: the fixed cost)
# and the stepping wave's phase stamps (-DCOG_STAMPS build) at the bench shard sizes.
#     tools/r05/gpu_probe.sh TAG
set -o pipefail
TAG=${1:-r05p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PROBE_SHORT=1 timeout -k 10 120 tools/r05/bin/duoprobe trio 65536 32768 16384 8192 > "$OUT/probe.txt" 2>&1 && \
PROBE_JSON=1 timeout -k 10 120 tools/r05/bin/duoprobe_st trio 65536 8192 > "$OUT/stamps.txt" 2>&1
rc=$?
cat "$OUT/probe.txt"; grep -v "^trio" "$OUT/stamps.txt" | head -60
exit $rc
