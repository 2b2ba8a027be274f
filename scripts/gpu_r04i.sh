#!/bin/bash
# Round 4: k_step_ag reading its kernel arguments per role (SGPR spills 44 -> 2): parity tests of
# the multi-wave kernels, then an interleaved A/B against the r03 build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04i
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_agents.py tests/test_gpu_parity.py tests/test_gpu_shards.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/ab_step.py 4096 12 build/libfjsp_r03.so multi-agent-rl-for-fjsp_amd/libfjsp.so build/libfjsp_r03.so multi-agent-rl-for-fjsp_amd/libfjsp.so > $OUT/ab_step.json 2> $OUT/ab_step.err
rc=$?; echo "ab rc=$rc"; python3 -c "import json; d=json.load(open('$OUT/ab_step.json')); [print(v['spec'], round(v['median_ms'],4), v['bytes_equal_to_first']) for v in d['variants']]"
exit 0
