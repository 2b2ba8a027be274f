#!/bin/bash
# Round 4: where the grouped update's time goes at HEAD (torch profiler, 4 096 and 32 768 envs:
# the latter is the gather exchange's learner), and the split-bf16 weight-gradient GEMM probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04e
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 200 python3 scripts/diag_wgrad_bf16.py > $OUT/wgrad_bf16.json 2> $OUT/wgrad_bf16.err
rc=$?; echo "wgrad rc=$rc"; cat $OUT/wgrad_bf16.json; tail -2 $OUT/wgrad_bf16.err; bad $rc && exit $rc
timeout -k 10 200 python3 scripts/prof_update_ops.py 4096 60 > $OUT/ops_4096.txt 2> $OUT/ops_4096.err
rc=$?; echo "ops 4096 rc=$rc"; head -30 $OUT/ops_4096.txt | cut -c1-200; bad $rc && exit $rc
timeout -k 10 300 python3 scripts/prof_update_ops.py 32768 60 > $OUT/ops_32768.txt 2> $OUT/ops_32768.err
rc=$?; echo "ops 32768 rc=$rc"; head -30 $OUT/ops_32768.txt | cut -c1-200
exit 0
