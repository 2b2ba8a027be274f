#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r04d.sh; rc=$?; echo "r04d rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04e.sh
