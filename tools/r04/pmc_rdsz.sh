#!/bin/bash
# Read bytes by request size (32 / 64 / 128 B) of the bench kernels, one rocprofv3 --pmc pass per
# shape, beside FETCH_SIZE: FETCH_SIZE's expression counts 128-B requests by TCC_BUBBLE, which on
# gfx950 misses wide reads (the guide's "double FETCH_SIZE" rule) -- exact bytes here instead.
#     tools/r04/pmc_rdsz.sh TAG
set -o pipefail
T=${1:-r04rd}
export TMPDIR=/tmp
BENCH="$PWD/bench.py"
run() {   # name, steps, chunk, envs
  local OUT=$PWD/gpurun_out/$T/$1
  mkdir -p "$OUT"
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/rd" -o run \
      --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
      -- python3 "$BENCH" --profile-steps "$2" --chunk "$3" --envs-total "$4" --warmup 0 --no-cpu-baseline) \
      > "$OUT/rd.log" 2>&1 && \
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/fetch" -o run \
      --pmc FETCH_SIZE -- python3 "$BENCH" --profile-steps "$2" --chunk "$3" --envs-total "$4" --warmup 0 --no-cpu-baseline) \
      > "$OUT/fetch.log" 2>&1 && \
  python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
}
run rd1000 2000 1000 65536 && run rd20_8192 200 20 8192
rc=$?
cat gpurun_out/$T/*/summary.txt | grep -E "^void|RDREQ|FETCH" 
exit $rc
