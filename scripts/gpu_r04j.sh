#!/bin/bash
# Round 4: k_step_pipe reading its kernel arguments per role (SGPR spills 25 -> 0 in the pre-draw
# build, 93 -> 32 without): parity tests of the multi-wave kernels, then the per-policy step
# costs against the build before the change, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_agents.py tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_config5.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; grep FAILED $OUT/pytest.log | head -3; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python3 scripts/diag_policies.py ../build/libfjsp_r04k.so 4096,65536 >> $OUT/policies.jsonl 2>> $OUT/policies.err || exit $?
  timeout -k 10 200 python3 scripts/diag_policies.py libfjsp.so 4096,65536 >> $OUT/policies.jsonl 2>> $OUT/policies.err || exit $?
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r04j/policies.jsonl"):
    r = json.loads(l); d[(r["N"], r["policy"], r["num_orders"], r["lib"])].append(r["us_per_step"])
keys = sorted({k[:3] for k in d})
for k in keys:
    print(k, "old", d[k + ("libfjsp_r04k.so",)], "new", d[k + ("libfjsp.so",)])
PY
