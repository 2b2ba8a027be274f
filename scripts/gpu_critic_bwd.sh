#!/bin/bash
# Fused critic backward in the grouped update: the critic test, the A2C tests, then the A2C bench
# with the fused backward, without it, and with neither fused pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-criticbwd}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_a2c.py -k fused_critic > $OUT/pytest0.log 2>&1 || exit $?
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_a2c.py tests/test_gpu_shards.py tests/test_gpu_config5.py > $OUT/pytest.log 2>&1 || exit $?
FJSP_CRITIC_BWD=1 timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_bwd1.json 2> $OUT/b1.err || exit $?
FJSP_CRITIC_BWD=0 timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_bwd0.json 2> $OUT/b0.err || exit $?
FJSP_CRITIC_FUSED=0 timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_none.json 2> $OUT/bn.err || exit $?
FJSP_CRITIC_BWD=1 timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_bwd1b.json 2> $OUT/b1b.err || exit $?
