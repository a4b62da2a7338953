#!/bin/bash
# build (here) or run (GPU box) the rollout timing tool (tools/ablate.cpp) under alternative
# compiler options (the production build uses max-ilp scheduling):
#     tools/flags_exp.sh build | tools/flags_exp.sh
set -o pipefail
M="-mllvm"
V=(ilp default clause ilp_nosink)
F=("$M -amdgpu-sched-strategy=max-ilp"
   ""
   "$M -amdgpu-sched-strategy=max-memory-clause"
   "$M -amdgpu-sched-strategy=max-ilp $M -sink-common-insts=false")
if [ "$1" = build ]; then
  for i in "${!V[@]}"; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off ${F[$i]} \
        -Iinclude -Igym-eldorado_amd/csrc tools/ablate.cpp -o tools/ablate_f_${V[$i]} &
  done
  wait
  for v in "${V[@]}"; do [ -x tools/ablate_f_$v ] || exit 1; done
  exit 0
fi
for v in "${V[@]}"; do
  printf "%-10s " $v; timeout -k 10 60 tools/ablate_f_$v 65536 3000 || exit 1
done
