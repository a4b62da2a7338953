#!/bin/bash
# Round-4 baseline on a fresh box: smoke, the driver's shape, the shard shapes (N = 1..8 sizes).
set -o pipefail
OUT=gpurun_out/${1:-r04a}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" && \
tools/gpu_shapes_r03e.sh "${1:-r04a}_shapes"
