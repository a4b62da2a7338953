#!/bin/bash
# The round's profiles (GPU box): rocprofv3 --kernel-trace --stats of the driver's bench command,
# then the PMC passes behind profiles/pmc_profile.json (instruction / cycle counts at 1,000-step
# launches; HBM traffic at the driver's 20-step launches and at 1,000).
#     tools/profile_round.sh TAG
set -o pipefail
TAG=${1:-prof}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$PWD
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
    -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras) > "$OUT/stats_bench.json" 2> "$OUT/stats.err" && \
tools/pmc_passes.sh "$TAG/pmc1000" 2000 1000 > /dev/null && \
tools/pmc_passes.sh "$TAG/pmc20" 100 20 > /dev/null
rc=$?
cat "$OUT/stats_bench.json"
find "$OUT/stats" -name "*kernel_stats.csv" | head -1 | xargs -r cat | head -20
exit $rc
