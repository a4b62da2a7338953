#!/bin/bash
# the full GPU test suite and smoke, as the round-end driver runs them
set -o pipefail
mkdir -p gpurun_out/r04hh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04hh/tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04hh/smoke.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04hh/tests.log; tail -n 1 gpurun_out/r04hh/smoke.log; exit $rc
