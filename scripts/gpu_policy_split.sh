#!/bin/bash
# Split-bf16 policy kernel: accuracy vs float64, timing, and the policy tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/polsplit
mkdir -p $OUT
timeout -k 10 300 python3 scripts/acc_policy.py 4096 random > $OUT/acc_random.json 2> $OUT/acc_random.err || exit $?
timeout -k 10 300 python3 scripts/acc_policy.py 4096 trained > $OUT/acc_trained.json 2> $OUT/acc_trained.err || exit $?
timeout -k 10 300 python3 scripts/ab_policy.py 4096 random multi-agent-rl-for-fjsp_amd/libfjsp.so multi-agent-rl-for-fjsp_amd/libfjsp.so::values multi-agent-rl-for-fjsp_amd/libfjsp.so::actors > $OUT/ab_random.json 2> $OUT/ab_random.err || exit $?
timeout -k 10 300 python3 scripts/ab_policy.py 4096 trained multi-agent-rl-for-fjsp_amd/libfjsp.so > $OUT/ab_trained.json 2> $OUT/ab_trained.err || exit $?
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_a2c.py tests/test_gpu_trained.py > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_a2c.json 2> $OUT/bench_a2c.err
