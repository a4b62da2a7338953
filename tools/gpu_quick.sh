#!/bin/bash
# Quick GPU iteration: parity tests, a short bench, the rollout phase-stamp diagnostic (if built).
#     tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 && \
timeout -k 10 200 python bench.py --steps 5000 --warmup 200 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" && \
{ [ ! -x tools/stamp_step ] || timeout -k 10 120 tools/stamp_step 65536 1 200 > "$OUT/stamp.txt" 2>&1; }
rc=$?
tail -3 "$OUT/tests.log"
python -c "import json;d=json.load(open('$OUT/bench.json'));print('value %.4g  us/step %.3f  kernel %.3f ms/launch  | per-launch %.4g  %.2f us' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms'], d['per_launch']['value'], d['per_launch']['kernel_ms']*1e3))" 2>/dev/null
cat "$OUT/stamp.txt" 2>/dev/null
exit $rc
