#!/bin/bash
# A/B of two engine builds on one box through tools/hostlat (device time of rollout(K) launches by
# HIP events, and the wall time of the calls): A = tools/abA/libcog_hip.so (tools/build_abA.sh),
# B = the tree's; alternated, ROUNDS times per size.
#     tools/gpu_ab_lib.sh TAG ROUNDS N...
set -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for n in "$@"; do
    LD_LIBRARY_PATH=$PWD/tools/abA timeout -k 10 120 tools/hostlat "$n" 20 > "$OUT/A_${n}_$r.txt" 2>&1 || exit 1
    timeout -k 10 120 tools/hostlat "$n" 20 > "$OUT/B_${n}_$r.txt" 2>&1 || exit 1
  done
done
for n in "$@"; do
  for ab in A B; do
    for r in $(seq 1 "$R"); do
      f="$OUT/${ab}_${n}_$r.txt"
      echo "$ab n=$n r$r: K=20 $(grep 'K=  20' "$f" | sed 's/ *K=  20 *//') | K=100 $(grep 'K= 100' "$f" | sed 's/ *K= 100 *//')"
    done
  done
done
