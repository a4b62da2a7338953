#!/bin/bash
# Same-box A/B of the current engine (tools/bin/duoprobe) against a baseline probe binary
# ($BASE, default tools/bin/duoprobe_r05: the round-5 engine; tools/bin/duoprobe_base: HEAD's,
# built from `git archive HEAD`), the current engine's launch timeline at the driver's shape
# (duoprobe_st), plus the driver's bench line.      tools/gpu_ab.sh TAG
set -o pipefail
TAG=${1:-r06ab}
BASE=${BASE:-duoprobe_r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2 3; do
  timeout -k 10 120 tools/bin/duoprobe trio 65536 8192 >> "$OUT/probe.txt" 2>&1 || exit 1
  timeout -k 10 120 tools/bin/$BASE base 65536 8192 >> "$OUT/probe.txt" 2>&1 || exit 1
done
PROBE_CHUNK=20 timeout -k 10 120 tools/bin/duoprobe_st trio 65536 > "$OUT/stamps_65536.txt" 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err"
rc=$?
cat "$OUT/probe.txt"
grep -A6 "launch timeline" "$OUT/stamps_65536.txt"
python -c "import json;d=json.loads(open('$OUT/bench_driver.json').read().strip().splitlines()[-1]);r=d['roofline'];print('driver', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), round(r['kernel_ms']*1e3,1))"
exit $rc
