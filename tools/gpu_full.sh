#!/bin/bash
# Full GPU check: every -m gpu test, the host-latency probe and the default bench line.
#     tools/gpu_full.sh TAG
set -o pipefail
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 && \
timeout -k 10 60 tools/hostlat 65536 20 > "$OUT/hostlat.txt" 2>&1 && \
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
grep -E "passed|failed|error" "$OUT/tests.log" | tail -3
cat "$OUT/hostlat.txt" 2>/dev/null
cat "$OUT/bench.json" 2>/dev/null
exit $rc
