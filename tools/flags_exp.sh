#!/bin/bash
# build (here) or run (GPU box) the rollout timing tool (tools/ablate.cpp) under alternative
# compiler scheduling options:  tools/flags_exp.sh build | tools/flags_exp.sh
set -o pipefail
V=(base ilp clause)
F=("" "-mllvm -amdgpu-sched-strategy=max-ilp" "-mllvm -amdgpu-sched-strategy=max-memory-clause")
if [ "$1" = build ]; then
  for i in "${!V[@]}"; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off ${F[$i]} -Iinclude -Igym-eldorado_amd/csrc \
        tools/ablate.cpp -o tools/ablate_f_${V[$i]} || exit 1
  done
  exit 0
fi
for v in "${V[@]}"; do
  printf "%-8s " $v; timeout -k 10 60 tools/ablate_f_$v 65536 3000 || exit 1
done
