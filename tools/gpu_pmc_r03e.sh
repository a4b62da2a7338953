#!/bin/bash
# PMC passes of the current engine for profiles/pmc_profile.json: 1,000-step and 20-step launches.
set -o pipefail
T=${1:-r03e}; tools/pmc_passes.sh $T/pmc1000 2000 1000 > /dev/null && tools/pmc_passes.sh $T/pmc20 200 20 > /dev/null
rc=$?
ls gpurun_out/$T/pmc1000 gpurun_out/$T/pmc20 | head -30
exit $rc
