#!/bin/bash
# The closing set of a round in one GPU call (the engine must be final: the profiles are keyed by
# its source hash, tools/pmc_profile.py engine_hash):
#   1. PMC passes of the trio at every bench launch shape -> gpurun_out/TAG/pmc_profile.json
#      (bench.py's roofline traffic: FETCH_SIZE x 2 + WRITE_SIZE per launch)
#   2. s_memtime phase stamps of the stepping wave at the same shapes -> stamps_profile.json
#      (bench.py's roofline.limiter; tools/stamps_profile.py), and the lone-wave instruction
#      costs (tools/chainprobe.hip -> chainprobe.txt: roofline.limiter.issue_frac)
#   3. GPU tests, smoke, the default bench (all extras + CPU baseline), the driver's shape, the
#      N = 2, 4, 8 shard shapes, rocprofv3 kernel stats of the driver's shape
# Then, in the container: copy pmc_profile.json and stamps_profile.json into profiles/, and run
# python tools/issue_frac.py --chain gpurun_out/TAG/chainprobe.txt --json profiles/issue_profile.json
#     tools/gpu_final.sh TAG           (probes: tools/build_probes.sh, chainprobe built beside them)
set -o pipefail
T=${1:-final}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
tools/pmc_passes.sh $T/pmc1000 2000 1000 65536 > /dev/null && \
tools/pmc_passes.sh $T/pmc20 200 20 65536 > /dev/null && \
tools/pmc_passes.sh $T/pmc20_32768 200 20 32768 > /dev/null && \
tools/pmc_passes.sh $T/pmc20_16384 200 20 16384 > /dev/null && \
tools/pmc_passes.sh $T/pmc20_8192 200 20 8192 > /dev/null && \
python tools/pmc_profile.py "$OUT/pmc1000:1000" "$OUT/pmc20:20" "$OUT/pmc20_32768:20:32768" \
   "$OUT/pmc20_16384:20:16384" "$OUT/pmc20_8192:20:8192" --coeff keep > "$OUT/pmc_profile.json" && \
cp "$OUT/pmc_profile.json" profiles/pmc_profile.json && \
for n in 65536 32768 16384 8192; do
  PROBE_JSON=1 PROBE_CHUNK=20 timeout -k 10 120 tools/bin/duoprobe_st trio $n > "$OUT/stamps_$n.txt" 2>&1 || exit 1
done && \
python tools/stamps_profile.py "$OUT"/stamps_*.txt > "$OUT/stamps_profile.json" && \
cp "$OUT/stamps_profile.json" profiles/stamps_profile.json && \
timeout -k 10 60 tools/bin/chainprobe > "$OUT/chainprobe.txt" 2>&1 && \
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
  python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline'];print('$f', '%.4g' % d['value'], d['ms_per_step'], r['rollout_kind'], round(r['kernel_ms']*1e3,1), r.get('frac'))" 2>/dev/null
done
grep -h "k_env" "$OUT"/prof/drv_kernel_stats.csv
exit $rc
