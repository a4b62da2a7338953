#!/bin/bash
# poll period of the drawing and storing waves' progress waits: s_sleep 2 (default) / 8 / 1
set -o pipefail
OUT=gpurun_out/${1:-r04cc}
mkdir -p "$OUT"
COG_ROLLOUT=duo timeout -k 10 200 tools/duoprobe s2 65536 8192 > "$OUT/s2.txt" 2>&1 && \
COG_ROLLOUT=duo timeout -k 10 200 tools/duoprobe_s8 s8 65536 8192 > "$OUT/s8.txt" 2>&1 && \
COG_ROLLOUT=duo timeout -k 10 200 tools/duoprobe_s1 s1 65536 8192 > "$OUT/s1.txt" 2>&1 && \
COG_ROLLOUT=duo timeout -k 10 200 tools/duoprobe s2b 65536 8192 > "$OUT/s2b.txt" 2>&1
rc=$?
cat "$OUT"/s2.txt "$OUT"/s8.txt "$OUT"/s1.txt "$OUT"/s2b.txt
exit $rc
