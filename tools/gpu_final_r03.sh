#!/bin/bash
# Round-3 final GPU set in one call: PMC passes of the engine (1,000- and 20-step launches) and
# profiles/pmc_profile.json from them (on the box, so the bench's roofline uses this engine's
# counters; regenerate it in the tree from the merged captures afterwards), then the closing set
# (tests, smoke, default bench, driver shape, rocprofv3 stats) and the shard-size shapes.
#     tools/gpu_final_r03.sh TAG
set -o pipefail
T=${1:-r03f}
tools/gpu_pmc_r03e.sh "$T" > /dev/null && \
python tools/pmc_profile.py "gpurun_out/$T/pmc1000:1000" "gpurun_out/$T/pmc20:20" --coeff keep > "gpurun_out/$T/pmc_profile.json" && \
tools/gpu_close_r03e.sh "$T" && \
tools/gpu_shapes_r03e.sh "${T}_shapes"
