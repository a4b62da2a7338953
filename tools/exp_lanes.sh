#!/bin/bash
mkdir -p gpurun_out/lanes
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lanes/tests.log 2>&1 || { tail -5 gpurun_out/lanes/tests.log; exit 1; }
tail -1 gpurun_out/lanes/tests.log
for cfg in "1 0" "2 0" "2 6000" "4 0" "4 3000" "8 0" "8 2000"; do
  set -- $cfg
  COG_RUNNER_LANES=$1 COG_RUNNER_STAGGER_NS=$2 timeout -k 10 60 python bench.py --steps 3000 --warmup 200 --no-cpu-baseline > gpurun_out/lanes/b_$1_$2.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lanes/b_$1_$2.json'));print('lanes $1 stagger $2: %.4g env-steps/s, %.2f us/step' % (d['value'], d['ms_per_step']*1e3))"
done
