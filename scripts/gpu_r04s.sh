#!/bin/bash
# Round 4: (1) gaps between the bench's launches with the library's per-launch hipEvents on / off;
# (2) the grouping by the library (radix sort + scan + scatter, ABI 8): A2C / config-5 / ABI
# tests, the A2C bench twice, the update's op profile at 4 096 and 32 768 envs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04s
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 scripts/ab_gaps.py 8 > $OUT/ab_gaps.json 2> $OUT/ab_gaps.err
rc=$?; echo "gaps rc=$rc"; bad $rc && exit $rc
python3 -c "import json; d=json.load(open('$OUT/ab_gaps.json')); print(d['wall_ms_per_launch_median'], d['event_ms_per_launch_median'])"
timeout -k 10 600 python -u -m pytest tests/test_gpu_a2c.py tests/test_gpu_config5.py tests/test_abi.py tests/test_gpu_shards.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head -3; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_a2c_$i.json 2> $OUT/bench_a2c_$i.err
  rc=$?; echo "bench $i rc=$rc"; bad $rc && exit $rc
  python3 -c "import json; d=[json.loads(l) for l in open('$OUT/bench_a2c_$i.json') if l.startswith('{')][-1]; a=d['a2c']; print(d['value'], a.get('update_ms_per_batch'), a.get('collect_ms_per_batch'))"
done
timeout -k 10 200 python3 scripts/prof_update_ops.py 4096 60 > $OUT/ops_4096.txt 2> $OUT/ops_4096.err
rc=$?; echo "ops rc=$rc"; grep "Self CUDA time total" $OUT/ops_4096.txt; bad $rc && exit $rc
timeout -k 10 400 python3 scripts/prof_update_ops.py 32768 60 > $OUT/ops_32768.txt 2> $OUT/ops_32768.err
rc=$?; echo "ops32k rc=$rc"; grep "Self CUDA time total" $OUT/ops_32768.txt
exit 0
