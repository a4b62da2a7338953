#!/bin/bash
# PMC passes over the benchmark workload (bench.py --profile-steps K): each counter group in its
# own rocprofv3 run with --kernel-trace only (never combined with sys/runtime traces), then a
# per-kernel summary.   Usage (on the GPU box): tools/pmc_passes.sh TAG [K] [chunk] [envs]
set -o pipefail
TAG=${1:-pmc}; STEPS=${2:-2000}; CHUNK=${3:-1000}; ENVS=${4:-65536}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$PWD/bench.py"
run() {   # name, counters...
  local name=$1; shift
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run \
      --pmc "$@" -- python3 "$BENCH" --profile-steps "$STEPS" --chunk "$CHUNK" --envs-total "$ENVS" --warmup 0 --no-cpu-baseline) \
      > "$OUT/$name.log" 2>&1
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run l2 TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE && \
run l2w TCC_WRITE_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum && \
run inst SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM
rc=$?
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
exit $rc
