#!/bin/bash
# Instruction-cache counters of the bench kernel: list the SQC counters this rocprofv3 offers,
# then one --pmc pass with the instruction-cache hit / miss counts (k_step_ag, 200-step launches).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/icache"
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1
echo "list rc=$?"
grep -i "SQC_ICACHE\|SQC_TC_INST\|SQ_IFETCH\|SQ_INSTS_WAVE\|SQ_WAIT_INST_ANY" "$OUT/avail.txt" | head -40
ARGS="--no-cpu-baseline --no-step-mode --no-a2c --no-scale --no-chunk-compare --steps 4 --warmup 2 --chunk 200"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -T -d "$OUT/p1" -o p1 --output-format csv -- python3 bench.py $ARGS > "$OUT/p1.log" 2>&1
echo "pmc rc=$?"; tail -3 "$OUT/p1.log"
exit 0
