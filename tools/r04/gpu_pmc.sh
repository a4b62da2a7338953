#!/bin/bash
# PMC passes of the current engine at every launch shape bench.py reports (profiles/pmc_profile.json
# `rollouts`): N=1 (65,536 envs) at 1,000- and 20-step launches, and the N = 2, 4, 8 shards
# (32,768 / 16,384 / 8,192 envs) at the driver's 20-step launches; then the profile itself.
#     tools/r04/gpu_pmc.sh TAG
set -o pipefail
T=${1:-r04p}
tools/pmc_passes.sh $T/pmc1000 2000 1000 65536 > /dev/null && \
tools/pmc_passes.sh $T/pmc20 200 20 65536 > /dev/null && \
tools/pmc_passes.sh $T/pmc20_32768 200 20 32768 > /dev/null && \
tools/pmc_passes.sh $T/pmc20_16384 200 20 16384 > /dev/null && \
tools/pmc_passes.sh $T/pmc20_8192 200 20 8192 > /dev/null && \
python tools/pmc_profile.py "gpurun_out/$T/pmc1000:1000" "gpurun_out/$T/pmc20:20" "gpurun_out/$T/pmc20_32768:20:32768" \
   "gpurun_out/$T/pmc20_16384:20:16384" "gpurun_out/$T/pmc20_8192:20:8192" --coeff keep > "gpurun_out/$T/pmc_profile.json"
rc=$?
ls gpurun_out/$T
exit $rc
