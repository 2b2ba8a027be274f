#!/bin/bash
# Diagnostic: us per step of the default kernel with subsets of its outputs not written.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for nl in "" "masks" "obs_i8,term,trunc,status" "obs_i32,obs_f32" "rewards" "obs_i32,obs_i8,obs_f32,masks,rewards,term,trunc,status"; do
  NULL_OUTS="$nl" timeout -k 10 60 python scripts/diag_time.py ${DIAG_N:-4096} 2>&1 | grep -v amdgpu.ids || exit 1
done
