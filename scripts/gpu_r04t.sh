#!/bin/bash
# Round 4: run sums by block scans (no serial walks): the grouping / run-sum / A2C / config-5
# tests, the A2C bench, the update's op profile at 4 096 and 32 768 envs, then the driver-form
# step bench (library per-launch events off).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04t
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_a2c.py tests/test_gpu_config5.py tests/test_gpu_shards.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head -3; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_a2c_$i.json 2> $OUT/bench_a2c_$i.err
  rc=$?; echo "bench $i rc=$rc"; bad $rc && exit $rc
  python3 -c "import json; d=[json.loads(l) for l in open('$OUT/bench_a2c_$i.json') if l.startswith('{')][-1]; a=d['a2c']; print(d['value'], a.get('update_ms_per_batch'), a.get('collect_ms_per_batch'))"
done
timeout -k 10 200 python3 scripts/prof_update_ops.py 4096 60 > $OUT/ops_4096.txt 2> $OUT/ops_4096.err
rc=$?; echo "ops rc=$rc"; grep "Self CUDA time total" $OUT/ops_4096.txt; bad $rc && exit $rc
timeout -k 10 400 python3 scripts/prof_update_ops.py 32768 60 > $OUT/ops_32768.txt 2> $OUT/ops_32768.err
rc=$?; echo "ops32k rc=$rc"; grep "Self CUDA time total" $OUT/ops_32768.txt; grep -E "k_run|k_group" $OUT/ops_32768.txt | cut -c1-62,140-200; bad $rc && exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json; d=[json.loads(l) for l in open('$OUT/bench.json') if l.startswith('{')][-1]; print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
exit $rc
