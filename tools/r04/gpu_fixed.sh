#!/bin/bash
# fixed cost of the trio launches: 1/2/5-step launches, and a kernel trace of 20-step launches
# (trio + k_env_fixup device times and the gap between them)
set -o pipefail
OUT=gpurun_out/${1:-r04g}
mkdir -p "$OUT"
export TMPDIR=/tmp
PROBE_SHORT=1 timeout -k 10 120 tools/duoprobe trio 8192 65536 > "$OUT/trio_fixed.txt" 2>&1 && \
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/$OUT/prof" -o trio \
   -- "$OLDPWD/tools/duoprobe" trio 8192) > "$OUT/prof.log" 2>&1
rc=$?
cat "$OUT"/*_fixed.txt
grep -h "k_env" "$OUT"/prof/trio_kernel_stats.csv
exit $rc
