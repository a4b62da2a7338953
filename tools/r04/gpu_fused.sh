#!/bin/bash
# the trio with the fix-up pass as a never-inlined call inside the launch (<= 16,384 envs) against
# two launches ($COG_TRIO_FUSED=0), then the GPU tests
set -o pipefail
OUT=gpurun_out/${1:-r04f2}
mkdir -p "$OUT"
PROBE_SHORT=1 timeout -k 10 120 tools/duoprobe fused 16384 8192 > "$OUT/fused.txt" 2>&1 && \
PROBE_SHORT=1 COG_TRIO_FUSED=0 timeout -k 10 120 tools/duoprobe split 16384 8192 > "$OUT/split.txt" 2>&1 && \
PROBE_SHORT=1 timeout -k 10 120 tools/duoprobe fused_b 16384 8192 > "$OUT/fused_b.txt" 2>&1 && \
PROBE_SHORT=1 COG_TRIO_FUSED=0 timeout -k 10 120 tools/duoprobe split_b 16384 8192 > "$OUT/split_b.txt" 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
cat "$OUT"/fused.txt "$OUT"/split.txt "$OUT"/fused_b.txt "$OUT"/split_b.txt
tail -n 2 "$OUT/tests.log"
exit $rc
