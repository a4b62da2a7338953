#!/bin/bash
# Round-3 GPU round trip: selected parity tests, the default bench (all extras + CPU baseline) and
# the driver's shape.  Each GPU step has its own time limit; steps are chained with &&.
#     tools/gpu_r03.sh TAG [pytest targets...]
set -o pipefail
TAG=${1:-r03}
shift
TESTS=${*:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread \
    > "$OUT/tests.log" 2>&1 && \
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/bench_driver.json" 2>&1
rc=$?
tail -3 "$OUT/tests.log"
python tools/summ.py "$OUT" 2>/dev/null
exit $rc
