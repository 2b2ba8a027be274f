#!/bin/bash
# Round-3 third session, final check at HEAD: smoke, every GPU test, the bench (driver defaults),
# the step kernels' rocprofv3 passes (trace, FETCH_SIZE, WRITE_SIZE), then the A2C loop's kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_r03.sh || exit $?
bash scripts/gpu_prof_a2c.sh > gpurun_out/prof_a2c.log 2>&1
echo "a2c prof rc=$?"
exit 0
