#!/bin/bash
# Round 4: k_step_ag allowed for 16 384 < N <= 32 768 (two rounds of 64-env workgroups): the
# multi-wave tests (with the new two-round case), the pre-draw tests, then the bench's scale leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04z
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_agents.py tests/test_gpu_predraw.py tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_config5.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_step.py 32768 8 build/libfjsp_r04l.so multi-agent-rl-for-fjsp_amd/libfjsp.so build/libfjsp_r04l.so multi-agent-rl-for-fjsp_amd/libfjsp.so > $OUT/ab_32768.json 2> $OUT/ab_32768.err
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$OUT/ab_32768.json')); [print(v['spec'], round(v['median_ms'],4), v['bytes_equal_to_first']) for v in d['variants']]"
