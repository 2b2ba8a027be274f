#!/bin/bash
# Round-3 profiling session: rocprofv3 kernel trace + stats and the HBM counter passes
# (FETCH_SIZE, WRITE_SIZE: one pass each) of the step bench (k_step_ag, k_step), the SQ passes of
# k_step_ag, and the A2C bench under the kernel trace (its JSON line kept) plus its counter passes
# (k_policy, k_step in the collect).  Each step under its own time limit; stops at the first
# timeout / fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 45; done ) &
HB=$!; trap 'kill $HB 2>/dev/null' EXIT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
bash scripts/gpu_profile.sh; rc=$?; echo "step profile rc=$rc"; bad $rc && exit $rc
bash scripts/gpu_pmc_sq.sh; rc=$?; echo "sq rc=$rc"; bad $rc && exit $rc
OUT="$PWD/gpurun_out/prof_a2c"
mkdir -p "$OUT"
A2C="--workload a2c --steps 4 --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py $A2C > "$OUT/kt.log" 2>&1
rc=$?; echo "a2c kt rc=$rc"; bad $rc && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -T -d "$OUT/$c" -o $c --output-format csv -- python3 bench.py $A2C > "$OUT/$c.log" 2>&1
  rc=$?; echo "a2c $c rc=$rc"; bad $rc && exit $rc
done
# the gather exchange's learner: one GPU running GAE + the update over 8 x 4 096 envs x 256 steps
timeout -k 10 300 python3 bench.py --workload a2c --envs 32768 --steps 3 --warmup 2 > "$OUT/a2c_32768envs.log" 2>&1
rc=$?; echo "a2c 32768 rc=$rc"; tail -c 600 "$OUT/a2c_32768envs.log"
exit 0
