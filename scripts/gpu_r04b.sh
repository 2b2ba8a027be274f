#!/bin/bash
# Round 4: the whole GPU suite (the graphed-update test first, then everything), each under a limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04b
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_a2c.py -k "graphed_update or policy_step" -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_first.log 2>&1
rc=$?; echo "first rc=$rc"; tail -4 $OUT/pytest_first.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" $OUT/pytest.log | tail -3; grep FAILED $OUT/pytest.log | head
exit $rc
