#!/bin/bash
# Round 4: k_step reading its outputs from the kernarg segment (SGPR spills 20 -> 0): the
# one-launch-per-step kernel's time per launch against the build before, and the tests that
# drive fjsp_step (parity, facade, edges).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04bb
mkdir -p $OUT
L="build/libfjsp_kstep_old.so multi-agent-rl-for-fjsp_amd/libfjsp.so"
timeout -k 10 300 python3 scripts/ab_kstep.py 4096 8 $L $L > $OUT/ab_kstep.json 2> $OUT/ab_kstep.err
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$OUT/ab_kstep.json')); [print(v['spec'], round(v['median_ms_per_launch']*1e3,2), 'us', v['bytes_equal_to_first']) for v in d['variants']]"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_facade.py tests/test_gpu_edges.py tests/test_gpu_predraw.py tests/test_gpu_a2c.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head -3
exit $rc
