#!/bin/bash
# A/B session: bench-kernel timing (r02 build vs current, xcd_map 0/1), fused policy timing on a
# real collect (random-init and trained weights), then the A2C / multi-rank GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 45; done ) &
HB=$!; trap 'kill $HB 2>/dev/null' EXIT
PK=multi-agent-rl-for-fjsp_amd
timeout -k 10 200 python scripts/ab_step.py 4096 10 $PK/libfjsp_r02.so $PK/libfjsp.so $PK/libfjsp_noxcd.so > gpurun_out/ab_step.json 2> gpurun_out/ab_step.err
rc=$?; echo "ab_step rc=$rc"; tail -c 1500 gpurun_out/ab_step.json; [ $rc -le 1 ] || exit $rc
for init in random trained; do
  timeout -k 10 200 python scripts/ab_policy.py 4096 $init $PK/libfjsp_r02.so $PK/libfjsp.so $PK/libfjsp_pf3.so $PK/libfjsp_pf4.so $PK/libfjsp_pf6.so $PK/libfjsp.so::actors $PK/libfjsp.so::values $PK/libfjsp_pf4.so::values > gpurun_out/ab_policy_$init.json 2>> gpurun_out/ab_policy.err
  rc=$?; echo "ab_policy $init rc=$rc"; tail -c 1500 gpurun_out/ab_policy_$init.json; [ $rc -le 1 ] || exit $rc
done
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_config5.py tests/test_gpu_shards.py tests/test_gpu_a2c.py tests/test_gpu_trained.py} -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu2.log
exit $rc
