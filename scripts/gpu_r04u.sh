#!/bin/bash
# Round 4 at HEAD: the gather learner by r03's method (A2C bench at 32 768 envs on one GPU = rank
# 0's GAE + update over 8 x 1.05 M samples), then the A2C kernel trace + counter passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04u
mkdir -p $OUT
bad() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 500 python3 bench.py --workload a2c --envs 32768 --steps 3 --warmup 2 > $OUT/bench_a2c_32768.json 2> $OUT/bench_a2c_32768.err
rc=$?; echo "bench32k rc=$rc"; bad $rc && exit $rc
python3 -c "import json; d=[json.loads(l) for l in open('$OUT/bench_a2c_32768.json') if l.startswith('{')][-1]; a=d['a2c']; print(d['value'], a.get('update_ms_per_batch'), a.get('collect_ms_per_batch'))"
P="$PWD/gpurun_out/prof_a2c"
rm -rf "$P"; mkdir -p "$P"
A2C="--workload a2c --steps 4 --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$P/kt" -o kt --output-format csv -- python3 bench.py $A2C > "$P/kt.log" 2>&1
rc=$?; echo "a2c kt rc=$rc"; bad $rc && exit $rc
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  d=$(echo $c | cut -d' ' -f1 | tr 'A-Z' 'a-z'); [ "$d" = "fetch_size" ] && d=fetch; [ "$d" = "write_size" ] && d=write; [ "$d" = "tcc_hit_sum" ] && d=hit
  timeout -s KILL 300 rocprofv3 --pmc $c -T -d "$P/$d" -o $d --output-format csv -- python3 bench.py $A2C > "$P/$d.log" 2>&1
  rc=$?; echo "a2c $c rc=$rc"; bad $rc && exit $rc
done
exit 0
