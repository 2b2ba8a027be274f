#!/usr/bin/env python3
"""A/B of a library-wide policy-launch option (fjsp_set_option(NULL, name, v), csrc/fjsp_policy.hip:
policy_xmap, policy_split, policy_dedup): one learner per value, each captured with
its value, replayed in alternation (256 x N per batch, ms per batch), and the rollout slabs
compared byte for byte across values after every batch (the options change which workgroup
computes what, never a value).

usage: python scripts/ab_collect_xmap.py [N] [reps] [values, e.g. 0+1+2] [option, default policy_xmap]"""
import importlib
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")


def main(n=4096, reps=10, orders=(0, 1, 2), init="random", T=256, option="policy_xmap"):
    learners = {}
    for x in orders:
        A.nat.check(A.nat.lib().fjsp_set_option(None, option.encode(), x))   # library-wide, read per launch
        L = A.VecMultiAgentA2C(V.FJSPVecEnv(n), batch_size=T, seed=3)
        if init == "trained":
            L.load_state_dicts(A.load_npz_weights(os.path.join(REPO, "tests", "golden", "trained_policy.npz")))
        L.reset(seeds=torch.arange(n), num_orders=25)
        for _ in range(3):       # eager, capture, replay (each captured with its own order)
            L.collect()
            L.roll_over()
        learners[x] = L
    torch.cuda.synchronize()
    ms = {x: [] for x in orders}
    equal = True
    for _ in range(reps):
        for x in orders:
            L = learners[x]
            t0 = time.perf_counter()
            L.collect()
            torch.cuda.synchronize()
            ms[x].append((time.perf_counter() - t0) * 1e3)
        b0 = learners[orders[0]]._bufs
        for x in orders[1:]:
            b = learners[x]._bufs
            equal &= all(torch.equal(b0[k], b[k]) for k in ("feats", "masks", "actions", "values", "rewards", "term",
                                                            "trunc", "status"))
        for x in orders:
            learners[x].roll_over()
    med = {x: sorted(v)[len(v) // 2] for x, v in ms.items()}
    return {"option": option, "envs": n, "batch": T, "init": init, "collect_ms_median": med, "collect_ms": ms,
            "slabs_equal_across_orders": bool(equal)}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    orders = tuple(int(x) for x in sys.argv[3].replace(",", "+").split("+")) if len(sys.argv) > 3 else (0, 1, 2)
    option = sys.argv[4] if len(sys.argv) > 4 else "policy_xmap"
    for init in ("random", "trained"):
        print(json.dumps(main(n, reps, orders, init, option=option)), flush=True)
