#!/bin/bash
# One policy-kernel iteration: A/B against a saved build, the stamps timeline, the policy tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-polround}
REF=${2:-multi-agent-rl-for-fjsp_amd/libfjsp_pol34.so}
D=multi-agent-rl-for-fjsp_amd
mkdir -p $OUT
timeout -k 10 300 python3 scripts/ab_policy.py 4096 random $REF $D/libfjsp.so $D/libfjsp.so::values $D/libfjsp.so::actors > $OUT/ab_random.json 2> $OUT/ab.err || exit $?
timeout -k 10 300 python3 scripts/diag_policy_stamps.py $D/libfjsp_pstamps.so all 32 > $OUT/stamps_all.json 2> $OUT/stamps.err || exit $?
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_a2c.py tests/test_gpu_trained.py > $OUT/pytest.log 2>&1 || exit $?
