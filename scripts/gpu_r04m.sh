#!/bin/bash
# Round 4: partial MT row copies, why slower: r04l (whole rows), v1full (range tracked, whole rows
# stored), vb (HEAD's buffer stores, all kept), va (HEAD + the next draw's first 64 words of both
# runs stored), HEAD (only the range).  Interleaved, k_step_ag 4096 envs, 1024-step launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04m
mkdir -p $OUT
L="build/libfjsp_r04l.so build/libfjsp_v1full.so build/libfjsp_vb.so build/libfjsp_va.so multi-agent-rl-for-fjsp_amd/libfjsp.so"
timeout -k 10 400 python3 scripts/ab_step.py 4096 8 $L $L > $OUT/ab_step.json 2> $OUT/ab_step.err
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$OUT/ab_step.json')); [print(v['spec'], round(v['median_ms'],4), v['bytes_equal_to_first']) for v in d['variants']]"
