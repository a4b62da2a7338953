#!/bin/bash
# Memory-pipeline counters of the rollout kernels (the store phase's cost): each counter group in
# its own rocprofv3 run with --kernel-trace only, over bench.py --profile-steps K at chunk K.
#   tools/pmc_stores.sh TAG KIND [K] [ENVS]   KIND = wave | duo | pipe (COG_ROLLOUT)
set -o pipefail
TAG=${1:-pmcst}; KIND=${2:-wave}; STEPS=${3:-200}; ENVS=${4:-65536}
OUT=$PWD/gpurun_out/$TAG/${KIND}_$ENVS
mkdir -p "$OUT"
export TMPDIR=/tmp COG_ROLLOUT=$KIND
BENCH="$PWD/bench.py"
run() {   # name, counters...
  local name=$1; shift
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run \
      --pmc "$@" -- python3 "$BENCH" --profile-steps "$STEPS" --chunk "$STEPS" --warmup 0 --no-cpu-baseline \
      --envs-total "$ENVS") \
      > "$OUT/$name.log" 2>&1
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_INSTS_VALU && \
run ta1 TA_TA_BUSY_sum TA_FLAT_WRITE_WAVEFRONTS_sum && \
run ta2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum && \
run tcp TCP_TCC_WRITE_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_ACCESSES_sum && \
run tcc TCC_WRITE_sum TCC_BUSY_sum TCC_TAG_STALL_sum TCC_REQ_sum && \
run tcc2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum && \
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
rc=$?
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
exit $rc
