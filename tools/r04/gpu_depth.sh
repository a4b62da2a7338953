#!/bin/bash
# trio ring depth 8 (default) against 4 (53.8 KB of LDS: three workgroups per CU)
set -o pipefail
OUT=gpurun_out/${1:-r04u}
mkdir -p "$OUT"
COG_ROLLOUT=duo timeout -k 10 200 tools/duoprobe d8 65536 49152 32768 16384 8192 > "$OUT/d8.txt" 2>&1 && \
COG_ROLLOUT=duo timeout -k 10 200 tools/duoprobe_d4 d4 65536 49152 32768 16384 8192 > "$OUT/d4.txt" 2>&1
rc=$?
cat "$OUT"/d8.txt "$OUT"/d4.txt
exit $rc
