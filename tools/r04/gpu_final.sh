#!/bin/bash
# Round-4 final set in one call: PMC passes of the engine at every bench launch shape and
# profiles/pmc_profile.json from them (written on the box, so the bench's roofline uses this
# engine's counters; copy gpurun_out/TAG/pmc_profile.json into profiles/ afterwards), then the
# closing set (tests, smoke, default bench, driver shape, shard shapes, rocprofv3 stats).
#     tools/r04/gpu_final.sh TAG
set -o pipefail
T=${1:-r04z}
bash tools/r04/gpu_pmc.sh "$T" > /dev/null && \
bash tools/r04/gpu_close.sh "$T"
