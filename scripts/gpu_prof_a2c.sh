#!/bin/bash
# Kernel-trace + stats of the A2C training-loop bench (collect via hipGraph + update).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/prof_a2c"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py --workload a2c --steps 2 --warmup 1 > "$OUT/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; tail -c 1500 "$OUT/kt.log"
head -40 "$OUT/kt/kt_kernel_stats.csv"
exit $rc
