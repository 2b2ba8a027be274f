#!/bin/bash
# Round 4: the fused collect with the tile state prefetched into LDS — its tests, the collect A/B,
# then the profiling passes (step bench + A2C bench: kernel trace, HBM bytes, L2 hit rate).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04d
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_a2c.py -k "policy_step or config4 or learn_matches or trained" -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/diag_collect.py 4096 > $OUT/collect_ab.json 2> $OUT/collect_ab.err
rc=$?; echo "collect ab rc=$rc"; cut -c1-300 $OUT/collect_ab.json; bad $rc && exit $rc
bash scripts/gpu_r04_prof.sh
