#!/bin/bash
# Round-3 closing set: GPU tests, smoke, the default bench (all extras + CPU baseline), the
# driver's shape, and rocprofv3 kernel stats of the driver's shape.  Each GPU step has its own
# time limit; steps are chained with &&.
#     tools/gpu_close_r03e.sh TAG
set -o pipefail
TAG=${1:-r03e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > "$OUT/tests.log" 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 500 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" && \
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/$OUT/prof" -o drv \
   -- python3 "$OLDPWD/bench.py" --steps 20 --warmup 5 --no-cpu-baseline) > "$OUT/prof.log" 2>&1
rc=$?
tail -3 "$OUT/tests.log"
tail -2 "$OUT/smoke.log"
python tools/summ.py "$OUT" 2>/dev/null
exit $rc
