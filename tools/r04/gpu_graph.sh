#!/bin/bash
# graph A/B of the driver's call shape (tools/r04/call_wall.py), then the rollout GPU tests
set -o pipefail
OUT=gpurun_out/${1:-r04x}
mkdir -p "$OUT"
COG_NO_GRAPH=1 timeout -k 10 200 python -u tools/r04/call_wall.py > "$OUT/plain.txt" 2>&1 && \
timeout -k 10 200 python -u tools/r04/call_wall.py > "$OUT/graph.txt" 2>&1 && \
COG_NO_GRAPH=1 timeout -k 10 200 python -u tools/r04/call_wall.py > "$OUT/plain2.txt" 2>&1 && \
timeout -k 10 200 python -u tools/r04/call_wall.py > "$OUT/graph2.txt" 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
tail -n 1 "$OUT"/plain.txt "$OUT"/graph.txt "$OUT"/plain2.txt "$OUT"/graph2.txt
tail -n 2 "$OUT/tests.log"
exit $rc
