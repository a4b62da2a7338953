#!/bin/bash
# A/B of engine environment overrides on chosen shapes (wall clock per 20-step call, kernel time).
#     tools/r05/gpu_ab.sh TAG "65536 8192" "base:X=1" "jt0:COG_TRIO_JT=0" ...
set -o pipefail
TAG=$1; SHAPES=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for n in $SHAPES; do
  for rep in 1 2; do
    for v in "$@"; do
      lab=${v%%:*}; envs=${v#*:}
      env $envs timeout -k 10 120 python bench.py --envs-total $n --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
        > "$OUT/$lab.$n.$rep.json" 2> "$OUT/$lab.$n.$rep.err" || exit 1
      python -c "import json;d=json.loads(open('$OUT/$lab.$n.$rep.json').read().strip().splitlines()[-1]);print('%-10s %6d %.4g  %.3f us/step  kernel %.1f us' % ('$lab', $n, d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3))"
    done
  done
done
