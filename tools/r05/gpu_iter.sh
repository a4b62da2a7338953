#!/bin/bash
# One iteration: trio parity tests (rollout, timed workloads, configs, golden), then the probe
# timings and stamps.
#     tools/r05/gpu_iter.sh TAG [pytest -k EXPR]
set -o pipefail
TAG=${1:-r05i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
K=${2:-"trio or timed or rollout or golden or configs or horizon or views or parity"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > "$OUT/tests.log" 2>&1 && \
PROBE_SHORT=1 timeout -k 10 120 tools/r05/bin/duoprobe trio 65536 8192 > "$OUT/probe.txt" 2>&1 && \
for v in tools/r05/bin/duoprobe_v*; do
  [ -x "$v" ] || continue
  timeout -k 10 120 "$v" "$(basename "$v")" 65536 8192 >> "$OUT/probe.txt" 2>&1 || exit 1
done && \
PROBE_JSON=1 timeout -k 10 120 tools/r05/bin/duoprobe_st trio 65536 8192 > "$OUT/stamps.txt" 2>&1 && \
PROBE_JSON=1 PROBE_CHUNK=20 timeout -k 10 120 tools/r05/bin/duoprobe_st trio 65536 8192 > "$OUT/stamps20.txt" 2>&1
rc=$?
tail -n 3 "$OUT/tests.log"; cat "$OUT/probe.txt"; grep -A40 "stepping wave" "$OUT/stamps.txt" | head -70
grep STAMPS_JSON "$OUT/stamps20.txt"
exit $rc
