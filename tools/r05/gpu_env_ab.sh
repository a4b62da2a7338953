#!/bin/bash
# A/B of HIP runtime settings on the driver's shape (wall clock per 20-step call).
#     tools/r05/gpu_env_ab.sh TAG
set -o pipefail
TAG=${1:-r05env}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {   # label, env...
  local lab=$1; shift
  for rep in 1 2; do
    env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/$lab.$rep.json" 2> "$OUT/$lab.$rep.err" || return 1
    python -c "import json;d=json.loads(open('$OUT/$lab.$rep.json').read().strip().splitlines()[-1]);print('%-28s %.4g  %.3f us/step  kernel %.1f us' % ('$lab', d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3))"
  done
}
run base X=1 && run active_wait ROC_ACTIVE_WAIT_TIMEOUT=1000 && run dev_kernarg HIP_FORCE_DEV_KERNARG=1 && \
run both ROC_ACTIVE_WAIT_TIMEOUT=1000 HIP_FORCE_DEV_KERNARG=1 && run kernarg0 HIP_FORCE_DEV_KERNARG=0
