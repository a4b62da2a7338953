#!/bin/bash
# build (here) or run (GPU box) the rollout timing tool (tools/ablate.cpp) under alternative
# compiler options (all on top of the production max-ilp scheduling):
#     tools/flags_exp.sh build | tools/flags_exp.sh
set -o pipefail
M="-mllvm"
V=(ilp phi8 phi16 phi48 spec phi16spec)
F=(""
   "$M -two-entry-phi-node-folding-threshold=8 $M -phi-node-folding-threshold=4"
   "$M -two-entry-phi-node-folding-threshold=16 $M -phi-node-folding-threshold=8"
   "$M -two-entry-phi-node-folding-threshold=48 $M -phi-node-folding-threshold=16"
   "$M -spec-exec-max-speculation-cost=40 $M -spec-exec-max-not-hoisted=10"
   "$M -two-entry-phi-node-folding-threshold=16 $M -phi-node-folding-threshold=8 $M -spec-exec-max-speculation-cost=40 $M -spec-exec-max-not-hoisted=10")
if [ "$1" = build ]; then
  for i in "${!V[@]}"; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp ${F[$i]} \
        -Iinclude -Igym-eldorado_amd/csrc tools/ablate.cpp -o tools/ablate_f_${V[$i]} &
  done
  wait
  for v in "${V[@]}"; do [ -x tools/ablate_f_$v ] || exit 1; done
  exit 0
fi
for v in "${V[@]}"; do
  printf "%-10s " $v; timeout -k 10 60 tools/ablate_f_$v 65536 3000 || exit 1
done
