#!/bin/bash
# Fused critic forward in the grouped update: tests, then the A2C bench with and without it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-critic}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_a2c.py -k fused_critic > $OUT/pytest0.log 2>&1
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_a2c.py tests/test_gpu_shards.py tests/test_gpu_config5.py tests/test_gpu_trained.py > $OUT/pytest.log 2>&1
for f in 1 0 1; do  # FJSP_CRITIC_BWD A/B below
  FJSP_CRITIC_FUSED=$f timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_a2c_fused$f.json 2> $OUT/bench_a2c_fused$f.err || exit $?
done
