#!/bin/bash
# A/B of the two-wave rollout (k_env_rollout_pipe) against the one-wave kernel at the strong-
# scaling shard sizes, alternated in separate processes on one box.   tools/exp_pipe.sh [ROUNDS]
set -o pipefail
for r in $(seq 1 "${1:-2}"); do
  for v in 0 32768; do
    echo "== COG_ROLLOUT_PIPE_MAX=$v"
    COG_ROLLOUT_PIPE_MAX=$v timeout -k 10 120 python -u tools/exp_nl.py 32768,16384,8192,256 64 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
