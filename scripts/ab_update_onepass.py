#!/usr/bin/env python3
"""A/B of the grouped update's critic: the one-pass kernel (fjsp_a2c_critic_fused, a2c_vec
critic_onepass_on = True) against the three-kernel path (forward kernel, per-sample loss through
autograd, value-head and backward kernels).  Two learners with the same seed collect the same
batches; their updates alternate, each timed (synchronised) and its gradients before clip / Adam
kept for the first batch; then the critic loss histories.  Prints JSON.

usage: python scripts/ab_update_onepass.py [N] [batches]"""
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
from tests.parity_util import grad_errors  # noqa: E402


def main(n=4096, batches=6):
    Ls = {}
    for mode in ("three_kernel", "onepass"):
        L = A.VecMultiAgentA2C(V.FJSPVecEnv(n), batch_size=256, seed=3)
        L.reset(seeds=torch.arange(n), num_orders=25)
        Ls[mode] = L
    ms = {m: [] for m in Ls}
    grads = {}
    for i in range(batches):
        for mode, L in Ls.items():
            A.critic_onepass_on = mode == "onepass"
            L.collect()
            if i == 0:
                L.grad_probe = lambda g, m=mode: grads.__setitem__(m, g)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            L.update()
            torch.cuda.synchronize()
            ms[mode].append((time.perf_counter() - t0) * 1e3)
            L.grad_probe = None
            L.roll_over()
    errs = grad_errors(grads["onepass"], grads["three_kernel"])
    res = {"envs": n, "batches": batches, "update_ms": ms,
           "update_ms_median_after_first2": {m: sorted(v[2:])[len(v[2:]) // 2] for m, v in ms.items()},
           "first_batch_rel_grad_diff_max": max(e for _, e in errs),
           "first_batch_rel_grad_diff": [[list(s), e] for s, e in errs],
           "critic_loss": {m: L.critic_loss_history for m, L in Ls.items()}}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:]))
