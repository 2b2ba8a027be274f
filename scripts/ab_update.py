"""A/B of the A2C update's host-side settings at N envs (batch 256): per variant a fresh learner
runs 3 warm-up batches then NB timed ones; synchronised update time per batch (median), collect
beside.  Variants: FJSP_GROUP_BUCKETS (group counts bucketed so GEMM shapes repeat) and the
BLAS library torch dispatches to (hipBLASLt or rocBLAS), and the graph-captured update
(VecMultiAgentA2C.graph_update).  (r03: buckets 11.90 against 11.83 ms exact, rocBLAS 13.49.)

usage: python scripts/ab_update.py [N] [batches]
"""
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 6
res = {"N": N, "batches": NB, "variants": []}
for buckets, blas, graphed in (("0", "hipblaslt", False), ("1", "hipblaslt", False), ("1", "hipblaslt", True)):
    os.environ["FJSP_GROUP_BUCKETS"] = buckets
    torch.backends.cuda.preferred_blas_library(blas)
    L = A.VecMultiAgentA2C(V.FJSPVecEnv(N), batch_size=256, seed=0)
    L.graph_update = graphed
    L.reset(seeds=torch.arange(N), num_orders=25)
    for _ in range(3):
        L.collect(); L.update(); L.roll_over()
    tc, tu = [], []
    for _ in range(NB):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        L.collect()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        L.update()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        L.roll_over()
        tc.append((t1 - t0) * 1e3)
        tu.append((t2 - t1) * 1e3)
    res["variants"].append({"group_buckets": buckets, "blas": blas, "graphed_update": graphed,
                            "graphs": len(L._ugraphs), "update_ms_median": float(np.median(tu)),
                            "update_ms": tu, "collect_ms_median": float(np.median(tc)),
                            "critic_loss_last": L.critic_loss_history[-1]})
    del L
    torch.cuda.empty_cache()
print(json.dumps(res))
