#!/bin/bash
# One GPU iteration after an engine change: all GPU parity tests, the fixed-cost probe, and the
# rollout's us/step at 65,536 and 8,192 envs (1,000-step launches and the driver's 20-step calls).
#     tools/gpu_iter.sh TAG
set -o pipefail
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 && \
timeout -k 10 120 bash tools/fixedcost.sh 65536 > "$OUT/fixedcost.txt" 2>&1 && \
timeout -k 10 200 python -u tools/exp_nl.py 65536,8192 64 > "$OUT/timing.txt" 2>&1 && \
timeout -k 10 120 python -u tools/exp_step.py 65536,8192 >> "$OUT/timing.txt" 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/bench20.json" 2> "$OUT/bench20.err"
rc=$?
tail -3 "$OUT/tests.log"
cat "$OUT/fixedcost.txt" "$OUT/timing.txt" 2>/dev/null | grep -v amdgpu.ids
python -c "import json;d=json.load(open('$OUT/bench20.json'));print('bench20 value %.4g  us/step %.3f' % (d['value'], d['ms_per_step']*1e3))" 2>/dev/null
exit $rc
