#!/bin/bash
# Round-4 closing set: GPU tests, smoke, the default bench (all extras + CPU baseline), the driver's
# shape, the driver's shape at the per-GPU shard sizes of N = 2, 4, 8, and rocprofv3 kernel stats
# of the driver's shape.  Each GPU step has its own time limit; steps are chained with &&.
#     tools/r04/gpu_close.sh TAG
set -o pipefail
TAG=${1:-r04w}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > "$OUT/tests.log" 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 500 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" && \
for n in 32768 16384 8192; do
  timeout -k 10 120 python bench.py --envs-total $n --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
      > "$OUT/shape_$n.json" 2> "$OUT/shape_$n.err" || exit 1
done && \
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/$OUT/prof" -o drv \
   -- python3 "$OLDPWD/bench.py" --steps 20 --warmup 5 --no-extras --no-cpu-baseline) > "$OUT/prof.log" 2>&1
rc=$?
tail -n 3 "$OUT/tests.log"
tail -n 2 "$OUT/smoke.log"
for f in "$OUT"/bench.json "$OUT"/bench_driver.json "$OUT"/shape_*.json; do
  python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline'];print('$f', '%.4g' % d['value'], d['ms_per_step'], r['rollout_kind'], round(r['kernel_ms']*1e3,1), round(r['frac'],3), r.get('counter_frac'))" 2>/dev/null
done
grep -h "k_env" "$OUT"/prof/drv_kernel_stats.csv
exit $rc
