#!/bin/bash
# trio vs duo A/B (same binary, $COG_TRIO=0 selects the duo), fixed cost, stamps, then the GPU tests.
set -o pipefail
OUT=gpurun_out/${1:-r04e}
mkdir -p "$OUT"
COG_TRIO=0 timeout -k 10 120 tools/duoprobe duo 8192 > "$OUT/duo.txt" 2>&1 && \
PROBE_SHORT=1 timeout -k 10 120 tools/duoprobe trio 16384 8192 > "$OUT/trio.txt" 2>&1 && \
COG_ROLLOUT=duo timeout -k 10 120 tools/duoprobe trio_forced 65536 32768 > "$OUT/trio_big.txt" 2>&1 && \
timeout -k 10 120 tools/duoprobe_st trio_st 8192 > "$OUT/trio_st.txt" 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
cat "$OUT"/duo.txt "$OUT"/trio.txt "$OUT"/trio_big.txt "$OUT"/trio_st.txt; tail -3 "$OUT/tests.log"
exit $rc
