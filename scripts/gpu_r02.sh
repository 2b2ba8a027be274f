#!/bin/bash
# Round-2 GPU session: smoke -> GPU parity tests -> bench (driver defaults) -> rocprofv3 passes
# (kernel trace + stats, FETCH_SIZE, WRITE_SIZE) of the bench at the driver's configuration.
# Stops at the first fault / timeout; plain test failures (exit 1) still let the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; ok $rc || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_PROF" ] && exit 0
bash scripts/gpu_profile.sh
