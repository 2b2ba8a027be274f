#!/bin/bash
# Policy-kernel workgroup timelines from the stamps build (scripts/diag_policy_stamps.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-polstamps}
mkdir -p $OUT
L=multi-agent-rl-for-fjsp_amd/libfjsp_pstamps.so
for part in all actors values; do
  timeout -k 10 300 python3 scripts/diag_policy_stamps.py $L $part 32 > $OUT/stamps_$part.json 2> $OUT/stamps_$part.err || exit $?
done
