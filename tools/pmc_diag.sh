#!/bin/bash
# Diagnostic PMC passes over the rollout (tools/ablate_base: 65,536 envs, 1,000-step launches).
set -o pipefail
OUT=$PWD/gpurun_out/pmcdiag; mkdir -p "$OUT"; export TMPDIR=/tmp
BIN=$PWD/tools/ablate_base
run() { local name=$1; shift
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run --pmc "$@" -- "$BIN" 65536 2000) > "$OUT/$name.log" 2>&1; }
run a SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_CYCLES_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES && \
run b SQ_INST_LEVEL_VMEM SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VSKIPPED SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAIT_INST_LDS
rc=$?
python3 tools/pmc_summary.py "$OUT" 2>&1 | grep -A20 "k_env_rollout"
exit $rc
