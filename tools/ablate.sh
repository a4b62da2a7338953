#!/bin/bash
# build (here) or run (GPU box) the ablation variants of tools/ablate.cpp (build also makes
# tools/stamp_step, the phase-stamp diagnostic)
set -o pipefail
if [ "$1" = build ] || [ "$1" = build-base ]; then
  vs="${ABL:-base DUPSAMPLE DUPENDTURN DUPDISCARD DUPDRAW DUPPLAY DUPUPDOBS}"; [ "$1" = build-base ] && vs=base
  for v in $vs; do
    f=""; [ $v != base ] && f="-DCOG_ABLATE_$v"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp $f -Iinclude -Igym-eldorado_amd/csrc \
        tools/ablate.cpp -o tools/ablate_$v &
  done
  wait
  for v in $vs; do [ -x tools/ablate_$v ] || exit 1; done
  [ "$1" = build-base ] && exit 0
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DCOG_STAMPS -Iinclude \
      -Igym-eldorado_amd/csrc tools/stamp_step.cpp -o tools/stamp_step || exit 1
  exit 0
fi
for v in ${ABL:-base DUPSAMPLE DUPENDTURN DUPDISCARD DUPDRAW DUPPLAY DUPUPDOBS}; do
  printf "%-8s " $v; timeout -k 10 60 tools/ablate_$v 65536 3000 || exit 1
done
