#!/bin/bash
# Builds the diagnostic probes (tools/duoprobe.cpp: plain and -DCOG_STAMPS) into tools/r06/bin/
# (git-ignored; they travel to the GPU box with the tree while present).
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/r06/bin
F="-O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp -Iinclude -Igym-eldorado_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F tools/duoprobe.cpp -o tools/r06/bin/duoprobe 2>/dev/null &
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -DCOG_STAMPS tools/duoprobe.cpp -o tools/r06/bin/duoprobe_st 2>/dev/null &
wait
