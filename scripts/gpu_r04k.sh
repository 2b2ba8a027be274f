#!/bin/bash
# Round 4: the pre-draw wave's row copy stores only the words the rows differ in (PG_SYNC):
# pre-draw / multi-wave parity tests, byte + time A/B of k_step_ag against the build before,
# then the step bench's kernel trace and FETCH / WRITE passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_predraw.py tests/test_gpu_agents.py tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_config5.py tests/test_gpu_edges.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/ab_step.py 4096 12 build/libfjsp_r04l.so multi-agent-rl-for-fjsp_amd/libfjsp.so build/libfjsp_r04l.so multi-agent-rl-for-fjsp_amd/libfjsp.so > $OUT/ab_step.json 2> $OUT/ab_step.err
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$OUT/ab_step.json')); [print(v['spec'], round(v['median_ms'],4), v['bytes_equal_to_first']) for v in d['variants']]"
bash scripts/gpu_profile.sh; rc=$?; echo "profile rc=$rc"
exit $rc
