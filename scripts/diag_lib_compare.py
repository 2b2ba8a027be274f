"""Timing of the step kernels in the library FJSP_LIB selects (default: the product build), for
comparing builds: k_step_ag launches of K = 1 .. 1024 steps (64 and 16 envs per workgroup),
k_step one launch per step, k_step_pipe with masked-random actions.  HIP-event times.

usage: FJSP_LIB=... python scripts/diag_lib_compare.py [N]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from tests import gpu_util as G  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
L = G.native.lib()
stream = torch.cuda.current_stream()


def timed(fn, reps):
    v = []
    for r in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        if r:
            v.append(e0.elapsed_time(e1) * 1e3)
    return float(np.median(v))


res = {"lib": os.path.basename(G.native.LIB_PATH), "N": N}
env = G.make_env(N)
env.reset(seeds=torch.arange(N))
b = G.vec_env.Buffers(1024, N, env.device, infos=False)
t = [0]


def roll(K, masked=False):
    def f():
        env.rollout(K, action_seed=3, step0=t[0], masked=masked, buffers=b)
        t[0] += K
    return f


for epw in (64, 16):
    G.native.check(L.fjsp_set_option(env.handle, b"ag_envs", epw))
    us = {K: timed(roll(K), 5) for K in (1, 2, 4, 20, 200, 1024)}
    Ks = np.array(list(us), float)
    slope, icpt = np.linalg.lstsq(np.stack([Ks, np.ones_like(Ks)], 1), np.array(list(us.values())), rcond=None)[0]
    res[f"ag_epw{epw}"] = {"us_per_launch": {int(k): round(v, 2) for k, v in us.items()},
                           "fit_us_per_step": round(float(slope), 4), "fit_intercept_us": round(float(icpt), 2),
                           "kernel": env.last_kernel()}
res["pipe_masked_1024_us"] = round(timed(roll(1024, True), 3), 1)
res["pipe_masked_kernel"] = env.last_kernel()
acts = (torch.randint(0, 1 << 16, (400, 8, N), device="cuda") %
        torch.tensor([3, 8, 3, 3, 3, 3, 3, 3], device="cuda").view(1, 8, 1)).to(torch.uint8)
sb = G.vec_env.Buffers(1, N, env.device, infos=False)
for i in range(20):
    env.step(acts[i], buffers=sb)
torch.cuda.synchronize()
ev = []
for i in range(20, 400):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    env.step(acts[i], buffers=sb)
    e1.record(stream)
    ev.append((e0, e1))
torch.cuda.synchronize()
res["k_step_us"] = round(float(np.median([a.elapsed_time(c) * 1e3 for a, c in ev])), 2)
res["k_step_kernel"] = env.last_kernel()
print(json.dumps(res), flush=True)
