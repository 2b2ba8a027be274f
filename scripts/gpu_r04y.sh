#!/bin/bash
# Round 4: k_step_ag (EPW 64, rounds of 256 workgroups) against k_step_pipe<1emit> above 16 384
# envs (diagnostic library build/libfjsp_ag64k.so: the agent-group kernel allowed up to 65 536
# envs), interleaved, outputs byte-compared.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04y
mkdir -p $OUT
for n in 32768 49152 65536 20480; do
  L="multi-agent-rl-for-fjsp_amd/libfjsp.so build/libfjsp_ag64k.so"
  timeout -k 10 300 python3 scripts/ab_step.py $n 8 $L $L > $OUT/ab_$n.json 2> $OUT/ab_$n.err
  rc=$?; echo "ab $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$OUT/ab_$n.json')); [print($n, v['spec'], round(v['median_ms'],4), round(v['min_ms'],4), v['bytes_equal_to_first']) for v in d['variants']]"
done
