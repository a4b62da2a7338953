#!/bin/bash
# Diagnostic: builds tools/fixedcost (base, no prologue player fill, no epilogue stores) on the
# CPU host; "run" on the GPU box prints each variant's per-launch device time against steps.
set -e
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp -Iinclude -Igym-eldorado_amd/csrc"
if [ "$1" = build ]; then
  for v in base FILL EPI FILL_EPI; do
    D=""; [ $v = FILL ] && D="-DCOG_ABLATE_FILL"; [ $v = EPI ] && D="-DCOG_ABLATE_EPI"
    [ $v = FILL_EPI ] && D="-DCOG_ABLATE_FILL -DCOG_ABLATE_EPI"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 $F $D tools/fixedcost.cpp -o tools/fixedcost_$v 2>/dev/null &
  done
  wait
  exit 0
fi
for v in base FILL EPI FILL_EPI; do
  echo "== $v n=${1:-65536}"
  timeout -k 10 60 tools/fixedcost_$v ${1:-65536}
done
