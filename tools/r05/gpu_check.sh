#!/bin/bash
# Round-5 iteration set: GPU tests (all, or a -k expression), the driver's shape (N=1), the N=2/4/8
# shard shapes, and rocprofv3 kernel stats of the driver's shape.  Each GPU step has its own limit.
#     tools/r05/gpu_check.sh TAG [pytest -k EXPR]
set -o pipefail
TAG=${1:-r05a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$OUT/tests.log" 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" && \
for n in 32768 16384 8192; do
  timeout -k 10 120 python bench.py --envs-total $n --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
      > "$OUT/shape_$n.json" 2> "$OUT/shape_$n.err" || exit 1
done && \
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/$OUT/prof" -o drv \
   -- python3 "$OLDPWD/bench.py" --steps 20 --warmup 5 --no-extras --no-cpu-baseline) > "$OUT/prof.log" 2>&1
rc=$?
tail -n 3 "$OUT/tests.log"
for f in "$OUT"/bench_driver.json "$OUT"/shape_*.json; do
  python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline'];print('$f', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), r['rollout_kind'], round(r['kernel_ms']*1e3,1))" 2>/dev/null
done
grep -h "k_env" "$OUT"/prof/drv_kernel_stats.csv
exit $rc
