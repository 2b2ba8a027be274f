#!/bin/bash
# Rehearsal of the multi-rank bench paths on a 1-GPU box: 2 ranks share the GPU, collectives on
# gloo (the driver's 8-GPU runs use one GPU per rank and RCCL).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export FJSP_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 400 --warmup 100 --no-cpu-baseline > gpurun_out/dist_step.log 2>&1
rc=$?; echo "dist step rc=$rc"; tail -c 1500 gpurun_out/dist_step.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29512 bench.py --gpus 2 --workload a2c --steps 2 --warmup 1 > gpurun_out/dist_a2c.log 2>&1
rc=$?; echo "dist a2c rc=$rc"; tail -c 1500 gpurun_out/dist_a2c.log
exit $rc
