#!/bin/bash
# Round-6 iteration: GPU tests (all, or a -k expression), then the driver's shape (N=1) with the
# multi-block trio on and off ($COG_TRIO_MB), twice each, interleaved, and the N=8 shard's shape.
#     tools/r06/gpu_iter.sh TAG [pytest -k EXPR]
set -o pipefail
TAG=${1:-r06x}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > "$OUT/tests.log" 2>&1 && \
for rep in 1 2; do
  for mb in 1 0; do
    COG_TRIO_MB=$mb timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
        > "$OUT/driver_mb${mb}_$rep.json" 2> "$OUT/driver_mb${mb}_$rep.err" || exit 1
  done
done && \
timeout -k 10 120 python bench.py --envs-total 8192 --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
    > "$OUT/shape_8192.json" 2> "$OUT/shape_8192.err"
rc=$?
tail -n 3 "$OUT/tests.log"
for f in "$OUT"/driver_*.json "$OUT"/shape_*.json; do
  python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline'];print('$f', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), r.get('rollout_kind'), round(r['kernel_ms']*1e3,1))" 2>/dev/null
done
exit $rc
