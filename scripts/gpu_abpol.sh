#!/bin/bash
# A/B of policy-kernel builds (scripts/ab_policy.py) on a real collect's observations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=multi-agent-rl-for-fjsp_amd
OUT=gpurun_out/${1:-polab}
mkdir -p $OUT
shift
timeout -k 10 300 python3 scripts/ab_policy.py 4096 random "$@" > $OUT/ab_random.json 2> $OUT/ab.err
