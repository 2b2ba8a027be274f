#!/bin/bash
# Round-3 GPU session: smoke -> GPU parity tests -> bench (driver defaults) -> optional rocprofv3
# passes.  A heartbeat file under gpurun_out/ shows progress during long tests (the 8-rank
# config-5 rehearsal prints nothing while its ranks run).  Stops at the first fault / timeout;
# plain test failures (exit 1) still let the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 45; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ -z "$NO_SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; ok $rc || exit $rc
fi
if [ -z "$NO_TESTS" ]; then
  FJSP_REPORT_DIR=gpurun_out/reports timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
fi
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_PROF" ] && exit 0
bash scripts/gpu_profile.sh
