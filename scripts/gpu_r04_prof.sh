#!/bin/bash
# Round-4 profiling: the step bench (kernel trace + FETCH_SIZE + WRITE_SIZE passes, gpu_profile.sh)
# and the A2C bench under the kernel trace (its JSON line kept) plus its counter passes (HBM bytes
# and the L2 hit rate of the collect's fused policy + step kernel).  Each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
bash scripts/gpu_profile.sh; rc=$?; echo "step profile rc=$rc"; bad $rc && exit $rc
OUT="$PWD/gpurun_out/prof_a2c"
mkdir -p "$OUT"
A2C="--workload a2c --steps 4 --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py $A2C > "$OUT/kt.log" 2>&1
rc=$?; echo "a2c kt rc=$rc"; bad $rc && exit $rc
i=0
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1)); d=$(echo $c | cut -d' ' -f1 | tr 'A-Z' 'a-z'); [ $i -eq 3 ] && d=hit; [ $i -eq 1 ] && d=fetch; [ $i -eq 2 ] && d=write
  timeout -s KILL 300 rocprofv3 --pmc $c -T -d "$OUT/$d" -o $d --output-format csv -- python3 bench.py $A2C > "$OUT/$d.log" 2>&1
  rc=$?; echo "a2c $c rc=$rc"; bad $rc && exit $rc
done
exit 0
