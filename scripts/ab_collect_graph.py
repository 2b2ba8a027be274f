#!/usr/bin/env python3
"""A/B of the collect's submission: the hipGraph replay of the whole batch against eager
launches on the env-group streams, for several group counts, one learner per variant, replayed
in alternation (256 x N per batch, ms per batch), the rollout slabs compared byte for byte
after every batch.

usage: python scripts/ab_collect_graph.py [N] [reps] [variants, e.g. g2,e1,e2,e3,e4]"""
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


def main(n=4096, reps=10, T=256, variants=("g2", "e2")):
    learners = {}
    for v in variants:
        L = A.VecMultiAgentA2C(V.FJSPVecEnv(n), batch_size=T, seed=3, use_graph=v[0] == "g")
        L.collect_groups = int(v[1:])
        L.reset(seeds=torch.arange(n), num_orders=25)
        for _ in range(3):
            L.collect()
            L.roll_over()
        learners[v] = L
    torch.cuda.synchronize()
    ms = {v: [] for v in variants}
    equal = True
    for _ in range(reps):
        for v in variants:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            learners[v].collect()
            torch.cuda.synchronize()
            ms[v].append((time.perf_counter() - t0) * 1e3)
        b0 = learners[variants[0]]._bufs
        for v in variants[1:]:
            b1 = learners[v]._bufs
            equal &= all(torch.equal(b0[k], b1[k]) for k in ("feats", "masks", "actions", "values", "rewards", "term",
                                                             "trunc", "status"))
        for L in learners.values():
            L.roll_over()
    med = {k: sorted(v)[len(v) // 2] for k, v in ms.items()}
    return {"envs": n, "batch": T, "variants": "g = hipGraph replay, e = eager; digit = env groups",
            "collect_ms_median": med, "collect_ms": ms, "slabs_equal": bool(equal)}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    variants = tuple(sys.argv[3].split(",")) if len(sys.argv) > 3 else ("g2", "e2")
    print(json.dumps(main(n, reps, variants=variants)), flush=True)
