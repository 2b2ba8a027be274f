#!/bin/bash
# Round-3 third session: the update's critic kernels on 64-sample tiles: the A2C GPU tests, A/B of
# the A2C bench (FJSP_CRITIC_TILE=64 / 32, alternating), the kernel trace of the A2C bench, the
# update's stage timing and torch-op profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ctile
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_a2c.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for t in 64 32; do
    FJSP_CRITIC_TILE=$t timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_${i}_tile$t.json 2> $OUT/bench_${i}_tile$t.err
    rc=$?; echo "bench $i tile=$t rc=$rc"; bad $rc && exit $rc
    python3 -c "import json; d=[json.loads(l) for l in open('$OUT/bench_${i}_tile$t.json') if l.startswith('{')][-1]; a=d['a2c']; print(d['value'], a.get('update_ms_per_batch'), a.get('collect_ms_per_batch'))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$PWD/$OUT/kt" -o kt --output-format csv -- python3 bench.py --workload a2c --steps 4 --warmup 3 > $OUT/kt.log 2>&1
rc=$?; echo "a2c kt rc=$rc"; bad $rc && exit $rc
timeout -k 10 300 python3 scripts/diag_update_stages.py 4096 > $OUT/stages.json 2> $OUT/stages.err
rc=$?; echo "stages rc=$rc"; bad $rc && exit $rc
timeout -k 10 300 python3 scripts/prof_update_ops.py 4096 60 > $OUT/ops.txt 2> $OUT/ops.err
echo "ops rc=$?"
exit 0
