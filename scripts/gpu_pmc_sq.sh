#!/bin/bash
# SQ counters (instruction mix, wave cycles) of the fused kernel, one pass per counter group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/sq"
mkdir -p "$OUT"
ARGS="--no-cpu-baseline --no-step-mode --no-a2c --no-scale --steps 400 --warmup 200 --chunk 200"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS" "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -T -d "$OUT/p$i" -o p$i --output-format csv -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
