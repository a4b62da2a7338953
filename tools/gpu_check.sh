#!/bin/bash
# GPU round-trip: parity tests, then the benchmark.  Each GPU step under its own time limit;
# steps chained with && so nothing runs after a failure.   Usage: tools/gpu_check.sh TAG [bench args]
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 400 python bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
cat gpurun_out/${TAG}_bench.json 2>/dev/null
exit $rc
