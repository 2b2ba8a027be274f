#!/bin/bash
# Round 4: k_step_ag A/B against r03 after the stall moved to its own instances; the update with
# the feature-row gathers back (A2C tests, benches, op profile).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04h
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 200 python3 scripts/ab_step.py 4096 12 build/libfjsp_r03.so multi-agent-rl-for-fjsp_amd/libfjsp.so build/libfjsp_r03.so multi-agent-rl-for-fjsp_amd/libfjsp.so > $OUT/ab_step.json 2> $OUT/ab_step.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_step.json; bad $rc && exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_a2c.py tests/test_gpu_config5.py tests/test_gpu_agents.py -k "not soak" -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head -3; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_a2c_$i.json 2> $OUT/bench_a2c_$i.err
  rc=$?; echo "bench $i rc=$rc"; bad $rc && exit $rc
  python3 -c "import json; d=[json.loads(l) for l in open('$OUT/bench_a2c_$i.json') if l.startswith('{')][-1]; a=d['a2c']; print(d['value'], a.get('update_ms_per_batch'), a.get('collect_ms_per_batch'))"
done
timeout -k 10 200 python3 scripts/prof_update_ops.py 4096 60 > $OUT/ops_4096.txt 2> $OUT/ops_4096.err
rc=$?; echo "ops rc=$rc"; grep "Self CUDA time total" $OUT/ops_4096.txt
exit 0
