#!/bin/bash
# Round 4 at HEAD: the k_step_ag soak (against k_step_pipe, every lean output bit for bit, five
# configurations, up to 2 000 steps on up to 16 384 envs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04w
mkdir -p $OUT
timeout -k 10 900 python3 -u scripts/soak_ag_parity.py > $OUT/soak_ag_parity.log 2>&1
rc=$?; echo "soak rc=$rc"; tail -6 $OUT/soak_ag_parity.log
exit $rc
