#!/bin/bash
# The two store costs behind bench.py's store roofline (GPU box): tools/storeprobe's packed pattern
# (scattered 16-B stores whose lines stay in L2: hits) and spread pattern (lines beyond an XCD's
# L2: mostly misses), timed without counters, then their L2 hits / misses per launch in a PMC pass.
#     tools/store_coeff.sh TAG        -> gpurun_out/TAG/{coeff.json, pmc/}
set -o pipefail
TAG=${1:-coeff}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 5 60 tools/storeprobe 65536 1 coeff > "$OUT/coeff.json" && \
(cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc" -o run \
    --pmc TCC_HIT_sum TCC_MISS_sum TCC_WRITE_sum TCC_EA0_WRREQ_sum -- "$OLDPWD/tools/storeprobe" 65536 1 coeff) \
    > "$OUT/pmc.log" 2>&1
rc=$?
cat "$OUT/coeff.json"
exit $rc
