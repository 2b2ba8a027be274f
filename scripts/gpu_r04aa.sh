#!/bin/bash
# Round 4: the grouping / run-sum kernels with their bounds guards: A2C and config-5 tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04aa
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_a2c.py tests/test_gpu_config5.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head -3
exit $rc
