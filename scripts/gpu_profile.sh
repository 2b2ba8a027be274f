#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then one PMC pass per
# TCC counter (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/prof"
mkdir -p "$OUT"
ARGS="${BENCH_ARGS:---no-cpu-baseline --no-a2c --no-scale --no-chunk-compare --no-dropin}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py $ARGS > "$OUT/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o fetch --output-format csv -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o write --output-format csv -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
rc=$?; echo "write rc=$rc"
find "$OUT" -name "*.csv" | head -20
exit $rc
