#!/bin/bash
# trio (forced) against the wave kernel over shard sizes: device us/step of 1,000- and 20-step launches
set -o pipefail
OUT=gpurun_out/${1:-r04p}
mkdir -p "$OUT"
COG_ROLLOUT=duo timeout -k 10 200 tools/duoprobe trio 65536 57344 49152 40960 32768 24576 > "$OUT/trio.txt" 2>&1 && \
COG_ROLLOUT=wave timeout -k 10 200 tools/duoprobe wave 65536 49152 32768 > "$OUT/wave.txt" 2>&1
rc=$?
cat "$OUT"/trio.txt "$OUT"/wave.txt
exit $rc
