#!/bin/bash
# k_step_ag diagnostics: per-wave stamps (diagnostic build) and A/B of build variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PK=multi-agent-rl-for-fjsp_amd
timeout -k 10 200 python scripts/diag_ag_stamps.py libfjsp_stamps.so 4096 > gpurun_out/ag_stamps.json 2> gpurun_out/ag_stamps.err
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/ag_stamps.json; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python scripts/ab_step.py 4096 10 $PK/libfjsp_r02.so $PK/libfjsp.so ${AB_VARIANTS} > gpurun_out/ab_step.json 2> gpurun_out/ab_step.err
rc=$?; echo "ab_step rc=$rc"; cat gpurun_out/ab_step.json
exit $rc
