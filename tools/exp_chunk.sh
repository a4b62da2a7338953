#!/bin/bash
# A/B of rollout steps per launch (COG_RUNNER_CHUNK) on the bench workload, after the parity tests.
mkdir -p gpurun_out/chunk
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chunk/tests.log 2>&1 || { tail -30 gpurun_out/chunk/tests.log; exit 1; }
tail -1 gpurun_out/chunk/tests.log
for c in 1 10 100 1000; do
  COG_RUNNER_CHUNK=$c timeout -k 10 60 python bench.py --steps 3000 --warmup 200 --no-cpu-baseline > gpurun_out/chunk/b_$c.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/chunk/b_$c.json'));print('chunk $c: %.4g env-steps/s, %.2f us/step, kernel %.2f us/step' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3))"
done
