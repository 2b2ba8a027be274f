"""A2C update time at N envs x 256 steps: dense (every sample through the networks) against
dedup (each network once per distinct input), after one collected batch; distinct-input counts.

usage: python scripts/diag_a2c_update.py [N] [dedup|dense|both]
"""
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
ve = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
which = sys.argv[2] if len(sys.argv) > 2 else "both"
out = {"N": N}
for dedup in ((False, True) if which == "both" else ((which == "dedup"),)):
    env = ve.FJSPVecEnv(N)
    L = A.VecMultiAgentA2C(env, seed=0, dedup=dedup)
    L.reset(seeds=torch.arange(N), num_orders=25)
    L.collect()
    ret, adv = L.advantages()
    L.update(ret, adv)          # warm-up (allocator, GEMM selection)
    torch.cuda.synchronize()
    ts = []
    for r in range(3):
        t0 = time.perf_counter()
        L.update(ret, adv)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    out["dedup" if dedup else "dense"] = {"update_ms": sorted(ts)[1], "all_ms": ts}
    if dedup:
        b = L._bufs
        x = A.actor_inputs(b["feats"][:L.batch_size], L.gidx)
        out["distinct_inputs"] = {a: int(A.group_columns(x[i]).first.numel()) for i, a in enumerate(A.AGENTS)}
        gt = b["feats"][:L.batch_size].permute(1, 0, 2).reshape(A.GLOBAL_DIM, -1)
        out["distinct_inputs"]["critic"] = int(A.group_columns(gt).first.numel())
        out["samples"] = int(x.shape[-1])
    del L, env
    torch.cuda.empty_cache()
print(json.dumps(out))
