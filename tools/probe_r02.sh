#!/bin/bash
# Round-2 baseline probe (GPU box): rollout us/step at the N=1 and N=8 shard sizes, the rollout
# phase stamps, and the bench at the driver's short length.   tools/probe_r02.sh TAG
set -o pipefail
TAG=${1:-probe}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
{ for n in 65536 32768 16384 8192 4096; do printf "%6d " $n; timeout -k 10 60 tools/ablate_base $n 3000 || exit 1; done; } > "$OUT/sizes.txt" 2>&1 && \
timeout -k 10 60 tools/stamp_step 65536 1 1000 > "$OUT/stamp65536.txt" 2>&1 && \
timeout -k 10 60 tools/stamp_step 8192 1 1000 > "$OUT/stamp8192.txt" 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench20.json" 2> "$OUT/bench20.err"
rc=$?
cat "$OUT/sizes.txt" "$OUT/stamp65536.txt" "$OUT/stamp8192.txt" 2>/dev/null
python -c "import json;d=json.load(open('$OUT/bench20.json'));print('bench20 value %.4g  us/step %.3f  kernel %.3f ms/launch' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms']))" 2>/dev/null
exit $rc
