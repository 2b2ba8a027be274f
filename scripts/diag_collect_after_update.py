#!/usr/bin/env python3
"""The collect's time after an update against after another collect (same learner, same box):
the bench's A2C loop times collect -> update -> roll_over, the option A/Bs collect -> roll_over.
Per batch: one collect right after an update, then one right after a collect (the update and the
collects all synchronised around), ms each; plus k_policy_step-free parts of the loop.

usage: python scripts/diag_collect_after_update.py [N] [reps]"""
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


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main(n=4096, reps=10, T=256):
    L = A.VecMultiAgentA2C(V.FJSPVecEnv(n), batch_size=T, seed=0)
    L.reset(seeds=torch.arange(n), num_orders=25)
    for _ in range(3):
        L.collect()
        L.update()
        L.roll_over()
    after_update, after_collect, update = [], [], []
    for _ in range(reps):
        after_update.append(timed(L.collect))
        L.roll_over()                              # that batch is dropped: no update between
        after_collect.append(timed(L.collect))
        update.append(timed(L.update))
        L.roll_over()
    med = lambda v: sorted(v)[len(v) // 2]   # noqa: E731
    return {"envs": n, "batch": T, "collect_ms_after_update_median": med(after_update),
            "collect_ms_after_collect_median": med(after_collect), "update_ms_median": med(update),
            "collect_ms_after_update": after_update, "collect_ms_after_collect": after_collect, "update_ms": update}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    print(json.dumps(main(n, reps)), flush=True)
