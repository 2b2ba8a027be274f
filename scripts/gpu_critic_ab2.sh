#!/bin/bash
# A2C bench order check: fused critic backward off / on / on / off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-criticab}
mkdir -p $OUT
i=0
for f in 0 1 1 0 1; do
  i=$((i+1))
  FJSP_CRITIC_BWD=$f timeout -k 10 300 python3 bench.py --workload a2c --steps 8 --warmup 4 > $OUT/bench_${i}_bwd$f.json 2> $OUT/b$i.err || exit $?
done
