#!/bin/bash
# duo A/B: base and new probes (us/step at 16,384 and 8,192; stamps), then the GPU parity tests.
set -o pipefail
OUT=gpurun_out/${1:-r04d}
mkdir -p "$OUT"
timeout -k 10 120 tools/duoprobe_base base 16384 8192 > "$OUT/duo_base.txt" 2>&1 && \
timeout -k 10 120 tools/duoprobe new 16384 8192 > "$OUT/duo_new.txt" 2>&1 && \
timeout -k 10 120 tools/duoprobe_base_st base_st 8192 > "$OUT/duo_base_st.txt" 2>&1 && \
timeout -k 10 120 tools/duoprobe_st new_st 8192 > "$OUT/duo_new_st.txt" 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
cat "$OUT"/duo_*.txt; tail -3 "$OUT/tests.log"
exit $rc
