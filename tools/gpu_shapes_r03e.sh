#!/bin/bash
# The driver's 20-step shape at the per-GPU shard sizes of N = 1, 2, 4, 8 (one GPU; 65,536 / N
# envs from global index 0), and rocprofv3 kernel stats of the N = 1 shape alone (no extras).
set -o pipefail
OUT=gpurun_out/${1:-r03e_shapes}
mkdir -p "$OUT"
export TMPDIR=/tmp
for n in 65536 32768 16384 8192; do
  timeout -k 10 120 python bench.py --envs-total $n --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
      > "$OUT/shape_$n.json" 2> "$OUT/shape_$n.err" || exit 1
  python -c "import json;d=json.loads(open('$OUT/shape_$n.json').read().strip().splitlines()[-1]);print('$n envs: %.4g env-steps/s  %.3f us/step  launch %.1f us' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3))"
done
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/$OUT/prof" -o drv \
   -- python3 "$OLDPWD/bench.py" --steps 20 --warmup 5 --no-extras --no-cpu-baseline) > "$OUT/prof.log" 2>&1
rc=$?
grep -h "k_env_rollout" "$OUT"/prof/drv_kernel_stats.csv
exit $rc
