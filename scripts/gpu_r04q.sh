#!/bin/bash
# Round 4: gaps between the bench's launches with the library's per-launch hipEvents on / off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04q
mkdir -p $OUT
timeout -k 10 300 python3 scripts/ab_gaps.py 8 > $OUT/ab_gaps.json 2> $OUT/ab_gaps.err
rc=$?; echo "gaps rc=$rc"; python3 -c "import json; d=json.load(open('$OUT/ab_gaps.json')); print(d['wall_ms_per_launch_median'], d['event_ms_per_launch_median'])"
exit $rc
