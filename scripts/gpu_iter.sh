#!/bin/bash
# Iteration loop on the GPU box: parity tests -> stamps -> quick perf.  Stops on faults.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for lib in ${STAMP_LIBS:-libfjsp_stamps.so}; do
  timeout -k 10 200 python scripts/diag_stamps.py $lib > gpurun_out/stamps_$lib.log 2>&1
  rc=$?; echo "stamps $lib rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps_$lib.log; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 200 python scripts/diag_perf.py ${DIAG_N:-4096,65536} > gpurun_out/diag.log 2>&1
rc=$?; echo "diag rc=$rc"; grep -v amdgpu.ids gpurun_out/diag.log
exit $rc
