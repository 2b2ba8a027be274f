#!/usr/bin/env python3
"""A/B of the A2C collect (diagnostic): fjsp_a2c_policy_step (policy + env step in one launch)
against fjsp_a2c_policy + fjsp_step (two launches per vector step), 256 x N per batch, the
captured graph replayed; alternating batches, ms per batch.  Prints JSON.

usage: python scripts/diag_collect.py [N] [group counts ...]"""
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


def main(n=4096, T=256, reps=8, init="random", groups=(1, 2, 4, 8)):
    learners = {}
    modes = [("g%d" % g, True, g) for g in groups] + [("two_launch", False, 1), ("g2_no_critic", True, 2)]
    for name, fused, g in modes:
        env = V.FJSPVecEnv(n)
        L = A.VecMultiAgentA2C(env, batch_size=T, seed=3)
        if init == "trained":
            L.load_state_dicts(A.load_npz_weights(os.path.join(REPO, "tests", "golden", "trained_policy.npz")))
        L.fused_step = fused
        L.collect_groups = g
        L._collect_values = name != "g2_no_critic"   # what the critic's workgroups cost the collect
        L.reset(seeds=torch.arange(n), num_orders=25)
        for _ in range(3):       # eager, capture, replay
            L.collect()
            L.roll_over()
        learners[name] = L
    torch.cuda.synchronize()
    ms = {name: [] for name, _, _ in modes}
    for _ in range(reps):
        for name, _, _ in modes:
            L = learners[name]
            t0 = time.perf_counter()
            L.collect()
            torch.cuda.synchronize()
            ms[name].append((time.perf_counter() - t0) * 1e3)
            L.roll_over()
    med = {k: sorted(v)[len(v) // 2] for k, v in ms.items()}
    return {"envs": n, "batch": T, "init": init, "collect_ms_median": med, "collect_ms": ms,
            "us_per_vector_step": {k: v * 1e3 / T for k, v in med.items()},
            "modes": "gN: fjsp_a2c_policy_step over N env groups on N streams; two_launch: fjsp_a2c_policy + fjsp_step"}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    groups = tuple(int(g) for g in sys.argv[2:]) or (1, 2, 4, 8)
    for init in ("random", "trained"):
        print(json.dumps(main(n, init=init, groups=groups)), flush=True)
