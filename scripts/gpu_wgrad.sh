#!/bin/bash
# Round-3 third session: the critic weight-gradient kernel (fjsp_a2c_critic_wgrad): its tests and
# the A2C tests, A/B of the A2C bench (FJSP_CRITIC_WGRAD=1 / 0, alternating), then the kernel
# trace of the A2C bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/wgrad
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_a2c.py -m gpu -x -v -k "wgrad or critic" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; bad $rc && exit $rc
for i in 1 2; do
  for w in 1 0; do
    FJSP_CRITIC_WGRAD=$w timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_${i}_wgrad$w.json 2> $OUT/bench_${i}_wgrad$w.err
    rc=$?; echo "bench $i wgrad=$w rc=$rc"; bad $rc && exit $rc
    python3 -c "import json,sys; d=[json.loads(l) for l in open('$OUT/bench_${i}_wgrad$w.json') if l.startswith('{')][-1]; a=d['a2c']; print(d['value'], a.get('update_ms_per_batch'), a.get('collect_ms_per_batch'))"
  done
done
[ -n "$NO_PROF" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$PWD/$OUT/kt" -o kt --output-format csv -- python3 bench.py --workload a2c --steps 4 --warmup 3 > $OUT/kt.log 2>&1
rc=$?; echo "a2c kt rc=$rc"
exit 0
