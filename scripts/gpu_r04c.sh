#!/bin/bash
# Round 4: the collect's env groups on concurrent streams (A/B), the A2C tests, two A2C benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 200 python3 scripts/diag_collect.py 4096 > $OUT/collect_ab.json 2> $OUT/collect_ab.err
rc=$?; echo "collect ab rc=$rc"; cut -c1-700 $OUT/collect_ab.json; bad $rc && exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_a2c.py tests/test_gpu_shards.py tests/test_gpu_trained.py tests/test_gpu_config5.py tests/test_gpu_parity.py -k "not golden_traces" -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/diag_update_stages.py 4096 > $OUT/stages.json 2> $OUT/stages.err
rc=$?; echo "stages rc=$rc"; cat $OUT/stages.json; bad $rc && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_a2c_$i.json 2> $OUT/bench_a2c_$i.err
  rc=$?; echo "bench $i rc=$rc"; bad $rc && exit $rc
  python3 -c "import json; d=[json.loads(l) for l in open('$OUT/bench_a2c_$i.json') if l.startswith('{')][-1]; a=d['a2c']; print(d['value'], a.get('update_ms_per_batch'), a.get('collect_ms_per_batch'))"
done
exit 0
