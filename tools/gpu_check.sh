#!/bin/bash
# Round-6 iteration set: GPU tests (all, or a -k expression), the driver's shape (N=1), the N=8
# shard's shape, and the probe beside the round-5 engine's (same box).  Each GPU step has its own
# limit.      tools/gpu_check.sh TAG [pytest -k EXPR]
set -o pipefail
TAG=${1:-r06a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$OUT/tests.log" 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" && \
timeout -k 10 120 python bench.py --envs-total 8192 --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
    > "$OUT/shape_8192.json" 2> "$OUT/shape_8192.err" && \
for rep in 1 2; do
  timeout -k 10 120 tools/bin/duoprobe trio 65536 8192 >> "$OUT/probe.txt" 2>&1 || exit 1
  timeout -k 10 120 tools/bin/duoprobe_r05 trio_r05 65536 8192 >> "$OUT/probe.txt" 2>&1 || exit 1
done
rc=$?
tail -n 3 "$OUT/tests.log"
for f in "$OUT"/bench_driver.json "$OUT"/shape_*.json; do
  python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline'];print('$f', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), r.get('rollout_kind'), round(r['kernel_ms']*1e3,1))" 2>/dev/null
done
cat "$OUT/probe.txt" 2>/dev/null
exit $rc
