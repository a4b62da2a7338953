#!/bin/bash
# trio roles fixed per wave slot against rotated per workgroup (-DCOG_TRIO_ROT): does a CU's second
# workgroup put its stepping wave on the same SIMD as the first's?
set -o pipefail
OUT=gpurun_out/${1:-r04y}
mkdir -p "$OUT"
timeout -k 10 200 tools/duoprobe fixed 65536 32768 24576 16384 8192 > "$OUT/fixed.txt" 2>&1 && \
timeout -k 10 200 tools/duoprobe_rot rot 65536 32768 24576 16384 8192 > "$OUT/rot.txt" 2>&1
rc=$?
cat "$OUT"/fixed.txt "$OUT"/rot.txt
exit $rc
