#!/bin/bash
# A/B of two builds of the package through the host API (tools/exp_nl.py), alternated in separate
# processes on one box: A = tools/abA_pkg (a package built from another revision), B = the tree.
#     tools/ab_pkg.sh [ROUNDS] [SIZES]
set -o pipefail
for r in $(seq 1 "${1:-2}"); do
  echo "== A"; COG_PKG_ROOT=$PWD/tools/abA_pkg timeout -k 10 120 python -u tools/exp_nl.py "${2:-32768,16384,8192}" 64 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== B"; timeout -k 10 120 python -u tools/exp_nl.py "${2:-32768,16384,8192}" 64 2>&1 | grep -v amdgpu.ids || exit 1
done
