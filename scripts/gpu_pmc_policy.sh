#!/bin/bash
# SQ counter passes (one group per run) of the A2C bench (k_policy, k_step of the collect) and of
# the step bench (k_step_ag): MFMA busy, waits, LDS pressure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/sq2"
mkdir -p "$OUT"
A2C="--workload a2c --steps 2 --warmup 2"
STEP="--no-cpu-baseline --no-step-mode --no-a2c --no-scale --steps 4 --warmup 2 --chunk 200 --no-chunk-compare"
i=0
run() {   # $1 = bench args, $2 = counters
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $2 -T -d "$OUT/p$i" -o p$i --output-format csv -- python3 bench.py $1 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($2) rc=$rc"; return $rc
}
run "$A2C" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" || exit $?
run "$A2C" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES" || exit $?
run "$STEP" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU" || exit $?
exit 0
