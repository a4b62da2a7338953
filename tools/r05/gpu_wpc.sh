#!/bin/bash
# A/B of trio workgroups per CU ($COG_TRIO_WPC) at 65,536 / 32,768 envs, after the trio parity tests.
#     tools/r05/gpu_wpc.sh TAG
set -o pipefail
TAG=${1:-r05w}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
   -k "trio or timed or rollout or golden or configs or horizon" > "$OUT/tests.log" 2>&1 && \
PROBE_SHORT=1 timeout -k 10 120 tools/r05/bin/duoprobe trio 65536 32768 8192 > "$OUT/probe.txt" 2>&1 && \
for w in 1 3 4; do
  COG_TRIO_WPC=$w timeout -k 10 120 tools/r05/bin/duoprobe wpc$w 65536 >> "$OUT/probe.txt" 2>&1 || exit 1
done && \
PROBE_JSON=1 timeout -k 10 120 tools/r05/bin/duoprobe_st trio 65536 8192 > "$OUT/stamps.txt" 2>&1
rc=$?
tail -n 3 "$OUT/tests.log"; cat "$OUT/probe.txt"; grep STAMPS_JSON "$OUT/stamps.txt"
exit $rc
