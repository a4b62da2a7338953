#!/bin/bash
# Fast GPU iteration: parity tests, then the rollout time of tools/ablate_base (build both first:
# build_ext.build_all() and tools/ablate.sh build-base).   Usage: tools/iter.sh TAG
set -o pipefail
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 && \
timeout -k 10 60 tools/ablate_base 65536 3000 > "$OUT/time.txt" 2>&1
rc=$?
tail -3 "$OUT/tests.log"
cat "$OUT/time.txt"
exit $rc
