#!/bin/bash
# A/B of two engine builds on one box through the C-ABI host-loop probe (tools/hostloop, C2 shape
# and more): A = tools/abA/libcog_hip.so (tools/build_abA.sh), B = the tree's; alternated.
#     tools/gpu_ab_hostloop.sh TAG [ROUNDS] [N...]
set -o pipefail
TAG=${1:-abhl}; R=${2:-3}; shift 2; SIZES=${*:-256}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for n in $SIZES; do
    LD_LIBRARY_PATH=$PWD/tools/abA timeout -k 10 120 tools/hostloop "$n" > "$OUT/A_${n}_$r.txt" 2>&1 || exit 1
    timeout -k 10 120 tools/hostloop "$n" > "$OUT/B_${n}_$r.txt" 2>&1 || exit 1
    echo "r$r n=$n A: $(grep "^n=" "$OUT/A_${n}_$r.txt" | cut -d'|' -f1)"
    echo "r$r n=$n B: $(grep "^n=" "$OUT/B_${n}_$r.txt" | cut -d'|' -f1)"
  done
done
