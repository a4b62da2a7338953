#!/bin/bash
# Same-box A/B of the current engine against the round-5 engine (probe binaries), plus the
# driver's bench line.      tools/gpu_ab.sh TAG
set -o pipefail
TAG=${1:-r06ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2 3; do
  timeout -k 10 120 tools/bin/duoprobe trio 65536 8192 >> "$OUT/probe.txt" 2>&1 || exit 1
  timeout -k 10 120 tools/bin/duoprobe_r05 trio_r05 65536 8192 >> "$OUT/probe.txt" 2>&1 || exit 1
done
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err"
rc=$?
cat "$OUT/probe.txt"
python -c "import json;d=json.loads(open('$OUT/bench_driver.json').read().strip().splitlines()[-1]);r=d['roofline'];print('driver', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), round(r['kernel_ms']*1e3,1))"
exit $rc
