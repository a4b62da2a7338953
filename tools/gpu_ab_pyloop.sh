#!/bin/bash
# A/B of two engine builds through the Python host loops of bench.py (C2: sampler.sample(masks);
# env.step(actions) at 256 envs; C4 shard: runner.sample(); runner.step_sync() at 8,192):
# A = tools/abA/libcog_hip.so (LD_LIBRARY_PATH), B = the tree's; alternated ROUNDS times.
#     tools/gpu_ab_pyloop.sh TAG ROUNDS
set -o pipefail
OUT=gpurun_out/$1; R=${2:-3}
mkdir -p "$OUT"
run() {
  timeout -k 10 200 python - <<'PY'
import json, sys
sys.argv = ["bench.py"]
import bench
import city_of_gold as cg
c2 = bench.host_loop(cg, 256, cg.EASY, 0, 2000, False)
c4 = bench.host_loop(cg, 8192, cg.HARD, 0, 300, True)
print("C2 %.1f us  C4 shard %.1f us" % (c2["ms_per_step"] * 1e3, c4["ms_per_step"] * 1e3))
PY
}
for r in $(seq 1 "$R"); do
  echo "A r$r: $(LD_LIBRARY_PATH=$PWD/tools/abA run 2>/dev/null | tail -1)"
  echo "B r$r: $(run 2>/dev/null | tail -1)"
done
