#!/bin/bash
# Round 4 at HEAD: the driver-form bench line, then the step and A2C profiles (gpu_r04_prof.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_final
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/bench.json; bad $rc && exit $rc
rm -rf gpurun_out/prof gpurun_out/prof_a2c
bash scripts/gpu_r04_prof.sh; rc=$?; echo "prof rc=$rc"
exit $rc
