#!/bin/bash
# PMC passes of the current engine for profiles/pmc_profile.json: 1,000-step and 20-step launches.
set -o pipefail
tools/pmc_passes.sh r03e/pmc1000 2000 1000 > /dev/null && tools/pmc_passes.sh r03e/pmc20 200 20 > /dev/null
rc=$?
ls gpurun_out/r03e/pmc1000 gpurun_out/r03e/pmc20 | head -30
exit $rc
