#!/bin/bash
# Diagnostic: where a short trio launch's time goes -- stamps of 1-, 2-, 5- and 20-step launches at
# 8,192 and 65,536 envs (the stepping wave's phases, per launch).
#     tools/r05/gpu_short.sh TAG
set -o pipefail
TAG=${1:-r05s}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for k in 1 2 5 20; do
  PROBE_JSON=1 PROBE_CHUNK=$k timeout -k 10 120 tools/r05/bin/duoprobe_st trio 8192 65536 > "$OUT/stamps_$k.txt" 2>&1 || exit 1
done
PROBE_SHORT=1 timeout -k 10 120 tools/r05/bin/duoprobe trio 8192 > "$OUT/probe.txt" 2>&1
rc=$?
for k in 1 2 5 20; do echo "== chunk $k"; grep STAMPS_JSON "$OUT/stamps_$k.txt"; done; cat "$OUT/probe.txt"
exit $rc
