#!/bin/bash
# The round's closing GPU evidence (one call): parity tests, smoke(), the driver's bench command
# (full line: extras + CPU baseline), the default bench, then rocprofv3 kernel stats of the
# driver's command and the PMC passes at 1,000- and 20-step launches (tools/profile_round.sh).
#     tools/final_round.sh TAG
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 && \
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench20.json" 2> "$OUT/bench20.err" && \
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" && \
bash tools/profile_round.sh "$TAG/prof" > "$OUT/prof.log" 2>&1 && \
timeout -k 10 200 python -u tools/exp_nl.py 65536,32768,16384,8192 64 > "$OUT/shard_sizes.txt" 2>&1
rc=$?
tail -3 "$OUT/tests.log"
cat "$OUT/smoke.txt"
python -c "import json;d=json.load(open('$OUT/bench20.json'));print('bench20 %.4g env-steps/s  %.3f us/step' % (d['value'], d['ms_per_step']*1e3))" 2>/dev/null
exit $rc
