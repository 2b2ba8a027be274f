#!/bin/bash
# Round 4: k_step_ag with and without the status output stream (4 B per env-step of the 215 the
# bench writes), interleaved, 4096 envs, 1024-step launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p $OUT
L="multi-agent-rl-for-fjsp_amd/libfjsp.so multi-agent-rl-for-fjsp_amd/libfjsp.so:nostatus=1"
timeout -k 10 300 python3 scripts/ab_step.py 4096 12 $L $L > $OUT/ab_step.json 2> $OUT/ab_step.err
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$OUT/ab_step.json')); [print(v['spec'], round(v['median_ms'],4), v['bytes_equal_to_first']) for v in d['variants']]"
