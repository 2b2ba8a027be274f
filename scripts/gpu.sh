#!/bin/bash
# One GPU session script for every stage (replaces the per-session gpu_r0*.sh files):
#   bash scripts/gpu.sh <out-dir-name> <stage> [<stage> ...]
# stages:
#   suite             the whole -m gpu suite (one process), then smoke()
#   tests:<expr>      pytest -m gpu -k <expr> (',' for ' ')
#   bench             the driver-form bench line (N=1)
#   bench_a2c[:args]  bench.py --workload a2c (extra args after ':' with ',' for ' ')
#   py:<script,args>  python3 <script> <args> (',' for ' '), stdout to <stage-index>.json
#   pyenv:<VAR=VAL+..>:<script,args>  the same with environment variables
#   prof_step         the step bench's kernel trace + FETCH_SIZE / WRITE_SIZE passes
#   prof_a2c[:args]   the A2C bench's kernel trace + FETCH / WRITE / L2-hit passes
#   pmc:<ctr,..>:<script,args>  one counter pass over a python script
#   profenv:<VAR=VAL+..>:<script,args>  kernel trace + stats of a python script with environment variables
# Every GPU step runs under its own time limit; the script stops at the first failure, abort,
# segfault or time-out (nothing more runs on the GPU after one).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$PWD/gpurun_out/$1"; shift
mkdir -p "$OUT"
bad() { [ "$1" -ne 0 ]; }
i=0
for stage in "$@"; do
  i=$((i+1))
  name="${stage%%:*}"; arg="${stage#*:}"; [ "$arg" = "$stage" ] && arg=""
  args="${arg//,/ }"
  echo "== stage $i: $stage"
  case "$name" in
    suite)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
      rc=$?; tail -3 "$OUT/pytest.log"; grep -E "FAILED|ERROR" "$OUT/pytest.log" | head -5
      bad $rc && exit $rc
      timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; tail -2 "$OUT/smoke.log" ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$args" > "$OUT/tests_$i.log" 2>&1
      rc=$?; tail -3 "$OUT/tests_$i.log"; grep -E "FAILED|ERROR" "$OUT/tests_$i.log" | head -5 ;;
    bench)
      timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
      rc=$?; tail -c 800 "$OUT/bench_$i.json" ;;
    bench_a2c)
      timeout -k 10 600 python3 bench.py --workload a2c $args > "$OUT/bench_a2c_$i.json" 2> "$OUT/bench_a2c_$i.err"
      rc=$?; tail -c 1200 "$OUT/bench_a2c_$i.json" ;;
    py)
      timeout -k 10 900 python3 -u $args > "$OUT/py_$i.json" 2> "$OUT/py_$i.err"
      rc=$?; tail -c 1500 "$OUT/py_$i.json"; [ $rc -ne 0 ] && tail -20 "$OUT/py_$i.err" ;;
    pyenv)
      # pyenv:VAR=VAL[+VAR=VAL]:script,args
      ev="${arg%%:*}"; rest="${arg#*:}"
      env ${ev//+/ } timeout -k 10 900 python3 -u ${rest//,/ } > "$OUT/py_$i.json" 2> "$OUT/py_$i.err"
      rc=$?; tail -c 1500 "$OUT/py_$i.json"; [ $rc -ne 0 ] && tail -20 "$OUT/py_$i.err" ;;
    prof_step)
      bash scripts/gpu_profile.sh; rc=$? ;;
    prof_a2c)
      A2C="--workload a2c --steps 4 --warmup 3 $args"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/a2c_kt" -o kt --output-format csv -- python3 bench.py $A2C > "$OUT/a2c_kt.log" 2>&1
      rc=$?; echo "a2c kt rc=$rc"; bad $rc && exit $rc
      for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
        d=$(echo "$c" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
        timeout -s KILL 300 rocprofv3 --pmc $c -T -d "$OUT/a2c_$d" -o $d --output-format csv -- python3 bench.py $A2C > "$OUT/a2c_$d.log" 2>&1
        rc=$?; echo "a2c $c rc=$rc"; bad $rc && exit $rc
      done ;;
    profenv)
      # profenv:VAR=VAL[+VAR=VAL]:script,args  kernel trace + stats of one python run
      ev="${arg%%:*}"; rest="${arg#*:}"
      env ${ev//+/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt_$i" -o kt --output-format csv -- python3 ${rest//,/ } > "$OUT/kt_$i.log" 2>&1
      rc=$? ;;
    pmc)
      ctr="${arg%%:*}"; rest="${arg#*:}"
      d=$(echo "${ctr%%,*}" | tr 'A-Z' 'a-z')_$i
      timeout -s KILL 300 rocprofv3 --pmc ${ctr//,/ } -T -d "$OUT/pmc_$d" -o pmc --output-format csv -- python3 ${rest//,/ } > "$OUT/pmc_$d.log" 2>&1
      rc=$? ;;
    *)
      echo "unknown stage $stage"; exit 2 ;;
  esac
  echo "== stage $i rc=$rc"
  bad $rc && exit $rc
done
exit 0
