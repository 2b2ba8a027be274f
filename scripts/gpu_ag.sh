#!/bin/bash
# k_step_ag bring-up: its own tests first, then timing of the default kernel vs the old one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_agents.py -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_ag.log 2>&1
rc=$?; echo "pytest ag rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_ag.log | head -30; [ $rc -le 1 ] || exit $rc
FJSP_AGENTS=1 timeout -k 10 120 python scripts/diag_time.py ${DIAG_N:-4096} 2>&1 | grep -v amdgpu.ids
rc=${PIPESTATUS[0]}; [ $rc -le 1 ] || exit $rc
FJSP_AGENTS=0 timeout -k 10 120 python scripts/diag_time.py ${DIAG_N:-4096} 2>&1 | grep -v amdgpu.ids
