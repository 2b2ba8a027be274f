#!/bin/bash
# LDS counters of the fused kernel (bank conflicts, LDS instruction cycles), one pass per group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/lds"
mkdir -p "$OUT"
ARGS="--no-cpu-baseline --no-step-mode --no-a2c --no-scale --steps 400 --warmup 200 --chunk 200"
i=0
for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS" "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -T -d "$OUT/p$i" -o p$i --output-format csv -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; grep -i "error" "$OUT/p$i.log" | head -3
  [ $rc -ge 124 ] && exit $rc
done
exit 0
