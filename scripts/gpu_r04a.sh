#!/bin/bash
# Round 4, first GPU call: bench.py --gpus 2 rehearsal (the driver's command form), the A2C tests,
# the update's stage timing and two A2C bench runs at HEAD (the r03 glue changes' GPU timing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 120 python3 scripts/diag_gae.py > $OUT/gae_ab.json 2> $OUT/gae_ab.err
rc=$?; echo "gae ab rc=$rc"; cat $OUT/gae_ab.json | cut -c1-600; bad $rc && exit $rc
timeout -k 10 120 python3 scripts/diag_collect.py 4096 > $OUT/collect_ab.json 2> $OUT/collect_ab.err
rc=$?; echo "collect ab rc=$rc"; cat $OUT/collect_ab.json | cut -c1-400; bad $rc && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_ranks.py tests/test_gpu_a2c.py tests/test_gpu_shards.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/diag_update_stages.py 4096 > $OUT/stages.json 2> $OUT/stages.err
rc=$?; echo "stages rc=$rc"; cat $OUT/stages.json; bad $rc && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_a2c_$i.json 2> $OUT/bench_a2c_$i.err
  rc=$?; echo "bench $i rc=$rc"; bad $rc && exit $rc
  python3 -c "import json; d=[json.loads(l) for l in open('$OUT/bench_a2c_$i.json') if l.startswith('{')][-1]; a=d['a2c']; print(d['value'], a.get('update_ms_per_batch'), a.get('collect_ms_per_batch'))"
done
exit 0
