#!/bin/bash
# Round-3 second session: the full GPU check (smoke, pytest -m gpu, bench), then the split-bf16
# policy kernel's accuracy and the A2C bench with its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
NO_PROF=1 bash scripts/gpu_r03.sh || exit $?
OUT=gpurun_out/r03b
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for init in random trained; do
  timeout -k 10 300 python3 scripts/acc_policy.py 4096 $init > $OUT/acc_$init.json 2> $OUT/acc_$init.err
  rc=$?; echo "acc $init rc=$rc"; bad $rc && exit $rc
done
timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_a2c.json 2> $OUT/bench_a2c.err
rc=$?; echo "a2c bench rc=$rc"; bad $rc && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$PWD/$OUT/kt" -o kt --output-format csv -- python3 bench.py --workload a2c --steps 4 --warmup 3 > $OUT/kt.log 2>&1
rc=$?; echo "a2c kt rc=$rc"
exit 0
