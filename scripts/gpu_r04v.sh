#!/bin/bash
# Round 4: the collect over 2 and 3 env groups (and 1), interleaved batches, random / trained init.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04v
mkdir -p $OUT
timeout -k 10 500 python3 -c "
import json, sys
sys.path.insert(0, 'scripts')
import diag_collect as D
for init in ('random', 'trained'):
    print(json.dumps(D.main(4096, init=init, groups=(1, 2, 3))), flush=True)
" > $OUT/collect_groups.jsonl 2> $OUT/collect_groups.err
rc=$?; echo "collect rc=$rc"; python3 -c "
import json
for l in open('$OUT/collect_groups.jsonl'): d=json.loads(l); print(d['init'], {k: round(v,3) for k,v in d['collect_ms_median'].items()})"
exit $rc
