mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_a2c.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_a2c.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_a2c.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 python scripts/ab_update.py 4096 12 > gpurun_out/ab_update.json 2> gpurun_out/ab_update.err; echo "ab rc=$?"; tail -5 gpurun_out/ab_update.err
python3 -c "import json; d=json.load(open('gpurun_out/ab_update.json')); [print(v['graphed_update'], v['graphs'], round(v['update_ms_median'],2), round(v['collect_ms_median'],2), v['critic_loss_last']) for v in d['variants']]"
