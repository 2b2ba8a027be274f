#!/bin/bash
# Round 4: k_step_ag at HEAD against the r03 build (interleaved 1 024-step launches), the driver's
# bench command, then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 200 python3 scripts/ab_step.py 4096 12 build/libfjsp_r03.so multi-agent-rl-for-fjsp_amd/libfjsp.so build/libfjsp_r03.so > $OUT/ab_step.json 2> $OUT/ab_step.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_step.json; bad $rc && exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/bench.json; bad $rc && exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" $OUT/pytest.log | tail -2; grep FAILED $OUT/pytest.log | head
exit $rc
