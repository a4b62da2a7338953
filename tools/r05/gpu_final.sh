#!/bin/bash
# Round-5 closing set in one call (the engine must be final: the profiles are keyed by its hash):
#   1. PMC passes of the trio at every bench launch shape -> profiles/pmc_profile.json (bench.py's
#      roofline traffic; tools/r04/gpu_pmc.sh)
#   2. s_memtime phase stamps of the stepping wave at the same shapes -> profiles/stamps_profile.json
#      (bench.py's roofline limiter; tools/r05/stamps_profile.py)
#   3. GPU tests, smoke, the default bench (all extras + CPU baseline), the driver's shape, the
#      N = 2, 4, 8 shard shapes, rocprofv3 kernel stats of the driver's shape (tools/r04/gpu_close.sh)
# Copy gpurun_out/TAG/{pmc_profile,stamps_profile}.json into profiles/ afterwards.
#     tools/r05/gpu_final.sh TAG
set -o pipefail
T=${1:-r05z}
OUT=gpurun_out/$T
mkdir -p "$OUT"
bash tools/r04/gpu_pmc.sh "$T" > "$OUT/pmc.log" 2>&1 && \
cp "$OUT/pmc_profile.json" profiles/pmc_profile.json && \
for n in 65536 32768 16384 8192; do
  PROBE_JSON=1 PROBE_CHUNK=20 timeout -k 10 120 tools/r05/bin/duoprobe_st trio $n > "$OUT/stamps_$n.txt" 2>&1 || exit 1
done && \
python tools/r05/stamps_profile.py "$OUT"/stamps_*.txt > "$OUT/stamps_profile.json" && \
cp "$OUT/stamps_profile.json" profiles/stamps_profile.json && \
bash tools/r04/gpu_close.sh "$T"
