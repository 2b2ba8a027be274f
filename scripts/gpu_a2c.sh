cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_a2c.py tests/test_gpu_policy_feats.py -x -q > gpurun_out/pytest_a2c.log 2>&1; rc=$?; tail -25 gpurun_out/pytest_a2c.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --workload a2c --steps 3 --warmup 1 > gpurun_out/bench_a2c.log 2>&1; rc=$?; tail -c 2500 gpurun_out/bench_a2c.log; exit $rc
