"""The bench's timed loop (k_step_ag, 4 096 envs, 1 024-step launches, one torch event pair per
launch) with the library's own per-launch hipEvents on and off (option "timing"): wall time per
launch including the gaps between launches, interleaved trials.

usage: python scripts/ab_gaps.py [trials]"""
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
TRIALS = int(sys.argv[1]) if len(sys.argv) > 1 else 6
N, K, L = 4096, 1024, 5
env = V.FJSPVecEnv(N)
env.reset(seeds=torch.arange(N), num_orders=30)
buf = V.Buffers(K, N, env.device, infos=False)
stream = torch.cuda.current_stream()
t = 0
res = {0: [], 1: []}
kern = {0: [], 1: []}
env.rollout(K, action_seed=1234, step0=t, buffers=buf)
t += K
for r in range(TRIALS):
    for lib_timing in (1, 0):
        nat.check(nat.lib().fjsp_set_option(env.handle, b"timing", lib_timing))
        torch.cuda.synchronize()
        ev = []
        t0 = time.perf_counter()
        for i in range(L):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            env.rollout(K, action_seed=1234, step0=t, buffers=buf)
            e1.record(stream)
            ev.append((e0, e1))
            t += K
        torch.cuda.synchronize()
        res[lib_timing].append((time.perf_counter() - t0) * 1e3 / L)
        kern[lib_timing].append(float(np.mean([a.elapsed_time(b) for a, b in ev])))
out = {"N": N, "K": K, "launches_per_trial": L,
       "wall_ms_per_launch_median": {f"lib_timing={k}": float(np.median(v)) for k, v in res.items()},
       "event_ms_per_launch_median": {f"lib_timing={k}": float(np.median(v)) for k, v in kern.items()},
       "wall": {str(k): v for k, v in res.items()}, "event": {str(k): v for k, v in kern.items()}}
print(json.dumps(out))
