#!/bin/bash
# Builds the diagnostic probes (tools/duoprobe.cpp: plain and -DCOG_STAMPS) and the lone-wave
# instruction-cost probe (tools/chainprobe.hip) into tools/bin/ (git-ignored; they travel to the
# GPU box with the tree while present).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
F="-O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp -falign-loops=64 -Iinclude -Igym-eldorado_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F tools/duoprobe.cpp -o tools/bin/duoprobe 2>/dev/null &
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -DCOG_STAMPS tools/duoprobe.cpp -o tools/bin/duoprobe_st 2>/dev/null &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/chainprobe.hip -o tools/bin/chainprobe 2>/dev/null
