#!/bin/bash
# GPU check of the host-loop paths: the parity tests, then the reference's numpy loop at C2
# (256 envs) through the C ABI (tools/hostloop) and through Python (bench.host_loop), with the
# completion-word spin (default) and with hipStreamSynchronize (COG_SPIN_US=0).
#     tools/gpu_hostloop.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-hostloop}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
  tail -2 "$OUT/tests.log"
fi
for spin in 2000 0; do
  COG_SPIN_US=$spin timeout -k 10 120 tools/hostloop 256 > "$OUT/hostloop_spin$spin.txt" 2>&1 || exit 1
  echo "spin=$spin C ABI: $(grep 'n=256' "$OUT/hostloop_spin$spin.txt")"
  COG_SPIN_US=$spin timeout -k 10 200 python - > "$OUT/pyloop_spin$spin.json" <<'EOF' || exit 1
import json, sys
sys.argv = ["bench.py"]
import bench
import city_of_gold as cg
print(json.dumps({"C2": bench.host_loop(cg, 256, cg.EASY, 0, 2000, False),
                  "C4_shard": bench.host_loop(cg, 8192, cg.HARD, 0, 200, True)}))
EOF
  python -c "import json;d=json.load(open('$OUT/pyloop_spin$spin.json'));print('spin=$spin python: C2 %.3g env-steps/s %.1f us/step; C4 shard %.3g %.1f us' % (d['C2']['value'], d['C2']['ms_per_step']*1e3, d['C4_shard']['value'], d['C4_shard']['ms_per_step']*1e3))"
done
