#!/bin/bash
# Diagnostic: instruction-cache counters of the rollout (bench workload, 1,000-step launches).
#     tools/icache_pmc.sh TAG
set -o pipefail
OUT=$PWD/gpurun_out/${1:-icache}
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$PWD/bench.py"
(cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ic" -o run \
    --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH \
    -- python3 "$BENCH" --profile-steps 2000 --chunk 1000 --warmup 0 --no-cpu-baseline) > "$OUT/ic.log" 2>&1
rc=$?
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
grep -A8 "k_env_rollout" "$OUT/summary.txt"
tail -5 "$OUT/ic.log"
exit $rc
