#!/bin/bash
# A/B of one environment switch on one box: tools/hostlat (device and wall time of rollout(K)
# launches) at the given shard sizes, alternating A (unset) and B (VAR=VALUE), twice each.
#     tools/gpu_ab_env.sh TAG VAR VALUE SIZE...
set -o pipefail
TAG=$1; VAR=$2; VAL=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for n in "$@"; do
    timeout -k 10 120 tools/hostlat "$n" 20 > "$OUT/A_${n}_$rep.txt" 2>&1 || exit 1
    env "$VAR=$VAL" timeout -k 10 120 tools/hostlat "$n" 20 > "$OUT/B_${n}_$rep.txt" 2>&1 || exit 1
  done
done
for n in "$@"; do
  for ab in A B; do
    for rep in 1 2; do
      f="$OUT/${ab}_${n}_$rep.txt"
      echo "$ab n=$n rep=$rep: $(head -1 "$f" | sed 's/.*device(events)/device/; s/, wall(rollout+streamsync).*//') | K=100 $(grep 'K= 100' "$f" | sed 's/ *K= 100 *//')"
    done
  done
done
