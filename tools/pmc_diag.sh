#!/bin/bash
# Diagnostic PMC passes (instruction fetch, branches, VMEM FIFO stalls, SALU/VALU issue) over the
# bench rollout.   Usage (GPU box): tools/pmc_diag.sh TAG [K] [chunk]
set -o pipefail
TAG=${1:-diag}; STEPS=${2:-2000}; CHUNK=${3:-1000}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$PWD/bench.py"
run() {
  local name=$1; shift
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run \
      --pmc "$@" -- python3 "$BENCH" --profile-steps "$STEPS" --chunk "$CHUNK" --warmup 0 --no-cpu-baseline) \
      > "$OUT/$name.log" 2>&1
}
run fetch_br SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VSKIPPED SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES && \
run vmem SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES && \
run issue SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
rc=$?
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
exit $rc
