#!/bin/bash
# Quick kernel iteration on the GPU box: rollout parity tests, rollout us/step at the N=1 and
# N=8 shard sizes (tools/ablate_base), and the bench at the driver's short length.
#     tools/quick_ab.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:-quick}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
T=${*:-tests/test_gpu_rollout.py}
timeout -k 10 600 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 && \
{ for n in 65536 8192; do printf "n %6d " $n; timeout -k 10 60 tools/ablate_base $n 3000 || exit 1; done; } > "$OUT/ab.txt" 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench20.json" 2> "$OUT/bench20.err"
rc=$?
tail -2 "$OUT/tests.log"; cat "$OUT/ab.txt"
python -c "import json;d=json.load(open('$OUT/bench20.json'));print('bench20 value %.4g  us/step %.3f  kernel %.3f ms/launch' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms']))" 2>/dev/null
exit $rc
