#!/bin/bash
# Same-box A/B of steady full dynamics (stored masks, 65,536 envs, the one-wave kernel) between the
# in-tree build and a copy of another build's package in tools/bin/base_pkg/city_of_gold (copy
# gym-eldorado_amd/city_of_gold there before rebuilding), then the GPU tests.
#     tools/fd_ab.sh            (profiles/r06_fd_stay_regs_ab.txt)
set -o pipefail
O=gpurun_out/r06fdab
mkdir -p $O
for r in 1 2; do
  COG_ROLLOUT=wave timeout -k 10 120 python tools/fd_kinds.py 65536 >> $O/ab.txt 2>&1 || exit 1
  COG_PKG=tools/bin/base_pkg COG_ROLLOUT=wave timeout -k 10 120 python tools/fd_kinds.py 65536 >> $O/ab.txt 2>&1 || exit 1
done
cat $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
exit $rc
