#!/bin/bash
# trio A/B against the duo ($COG_TRIO=0) and the wave kernel at 65,536; fixed cost, stamps, the C2
# host loop A/B, then the GPU tests.
set -o pipefail
OUT=gpurun_out/${1:-r04e}
mkdir -p "$OUT"
COG_TRIO=0 timeout -k 10 120 tools/duoprobe duo 8192 > "$OUT/duo.txt" 2>&1 && \
PROBE_SHORT=1 timeout -k 10 120 tools/duoprobe trio 16384 8192 > "$OUT/trio.txt" 2>&1 && \
COG_ROLLOUT=duo timeout -k 10 120 tools/duoprobe trio_forced 65536 32768 > "$OUT/trio_big.txt" 2>&1 && \
PROBE_SHORT=1 timeout -k 10 120 tools/duoprobe wave 65536 > "$OUT/wave.txt" 2>&1 && \
timeout -k 10 120 tools/duoprobe_st trio_st 8192 > "$OUT/trio_st.txt" 2>&1 && \
timeout -k 10 300 python -u tools/r04/c2_ab.py > "$OUT/c2.txt" 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
cat "$OUT"/duo.txt "$OUT"/trio.txt "$OUT"/trio_big.txt "$OUT"/wave.txt "$OUT"/trio_st.txt "$OUT"/c2.txt
tail -n 3 "$OUT/tests.log"
exit $rc
