#!/bin/bash
# Round 4: the update's glue ops by input shape and by Python stack (4 096 envs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04x
mkdir -p $OUT
timeout -k 10 300 python3 scripts/prof_update_shapes.py 4096 60 > $OUT/shapes_4096.txt 2> $OUT/shapes_4096.err
rc=$?; echo "shapes rc=$rc"; head -40 $OUT/shapes_4096.txt
exit $rc
