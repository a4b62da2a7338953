#!/bin/bash
# A/B timing of two engine versions on one box (tools/abprobe.cpp).
#   tools/ab.sh build [REV]   (here) A = the engine at git REV (default HEAD), B = the working tree
#   tools/ab.sh run [ROUNDS]  (GPU box) alternates A and B
set -o pipefail
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp"
if [ "$1" = build ]; then
  rm -rf /tmp/ab_a && mkdir -p /tmp/ab_a
  git archive "${2:-HEAD}" gym-eldorado_amd/csrc include | tar -x -C /tmp/ab_a || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -I/tmp/ab_a/gym-eldorado_amd/csrc -I/tmp/ab_a/include tools/abprobe.cpp -o tools/abprobe_A 2>/dev/null &
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -Igym-eldorado_amd/csrc -Iinclude tools/abprobe.cpp -o tools/abprobe_B 2>/dev/null &
  wait
  [ -x tools/abprobe_A ] && [ -x tools/abprobe_B ]
  exit $?
fi
for r in $(seq 1 "${2:-3}"); do
  timeout -k 10 60 tools/abprobe_A A || exit 1
  timeout -k 10 60 tools/abprobe_B B || exit 1
done
