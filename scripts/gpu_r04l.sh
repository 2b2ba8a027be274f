#!/bin/bash
# Round 4: partial MT row copies, variants A/B (k_step_ag 4096 envs, 1024-step launches):
# r04l = before, v1full = range tracked per refill but whole rows stored, HEAD = only the range
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04l
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_predraw.py tests/test_gpu_agents.py tests/test_gpu_parity.py tests/test_gpu_config5.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head -3; [ $rc -eq 0 ] || exit $rc
L="build/libfjsp_r04l.so build/libfjsp_v1full.so multi-agent-rl-for-fjsp_amd/libfjsp.so"
timeout -k 10 300 python3 scripts/ab_step.py 4096 10 $L $L > $OUT/ab_step.json 2> $OUT/ab_step.err
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$OUT/ab_step.json')); [print(v['spec'], round(v['median_ms'],4), v['bytes_equal_to_first']) for v in d['variants']]"
bash scripts/gpu_profile.sh; rc=$?; echo "profile rc=$rc"; exit $rc
