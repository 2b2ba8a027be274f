#!/bin/bash
# Timing of diagnostic library builds (VARIANT_LIBS) + stamps builds (STAMP_LIBS) on the GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in libfjsp.so ${VARIANT_LIBS}; do
  FJSP_LIB=$PWD/multi-agent-rl-for-fjsp_amd/$lib timeout -k 10 120 python scripts/diag_time.py ${DIAG_N:-4096} 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}; [ $rc -le 1 ] || exit $rc
done
for lib in ${STAMP_LIBS}; do
  timeout -k 10 200 python scripts/diag_stamps.py $lib > gpurun_out/stamps_$lib.log 2>&1
  rc=$?; echo "stamps $lib rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps_$lib.log | head -3; [ $rc -le 1 ] || exit $rc
done
