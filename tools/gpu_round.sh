#!/bin/bash
# One GPU round-trip: parity tests, the benchmark (with CPU baseline), a rocprofv3 kernel-trace
# --stats capture of a bench run, then the PMC passes.  Every GPU step has its own time limit and
# the steps are chained with && so nothing runs after a failure.
#     tools/gpu_round.sh TAG            (on the GPU box, from the repo root)
set -o pipefail
TAG=${1:-run}
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/tests.log" 2>&1 && \
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python3 "$ROOT/bench.py" --steps 2000 --warmup 1000 --no-cpu-baseline) \
    > "$OUT/prof_bench.json" 2> "$OUT/prof.err" && \
tools/pmc_passes.sh "$TAG/pmc" 2000
rc=$?
tail -3 "$OUT/tests.log"
cat "$OUT/bench.json" 2>/dev/null
cat "$OUT/prof_bench.json" 2>/dev/null
exit $rc
