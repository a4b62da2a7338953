#!/bin/bash
# the reference benchmark's horizon (10,200 steps) on the N=8 shard against the oracle
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_timed_workloads.py -k "10200" -v --timeout 650 --timeout-method thread > gpurun_out/r04gg_long.log 2>&1
rc=$?; tail -n 8 gpurun_out/r04gg_long.log; exit $rc
