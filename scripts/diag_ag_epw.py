"""k_step_ag with 64 / 32 / 16 envs per workgroup (option "ag_envs"): per-launch HIP-event time
at K = 1 .. 1024 steps (slope and intercept) and the outputs of a 1200-step run compared byte
for byte with the 64-env layout.

usage: python scripts/diag_ag_epw.py [N]
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
ref = None
res = {"N": N}
for epw in (64, 32, 16):
    env = G.make_env(N)
    G.native.check(L.fjsp_set_option(env.handle, b"ag_envs", epw))
    env.reset(seeds=torch.arange(N))
    # parity: 3 launches (600 + 400 + 200 steps) against the 64-env layout
    outs = []
    t = 0
    for K in (600, 400, 200):
        b = G.vec_env.Buffers(K, N, env.device, infos=False)
        env.rollout(K, action_seed=7, step0=t, buffers=b)
        t += K
        outs.append({k: v.copy() for k, v in G.to_np(b).items()})
    kern = env.last_kernel()
    if ref is None:
        ref = outs
        same = True
    else:
        same = all(a[k].tobytes() == r[k].tobytes() for a, r in zip(outs, ref) for k in r)
    b = G.vec_env.Buffers(1024, N, env.device, infos=False)
    ms = {}
    for K in (1, 2, 4, 8, 16, 20, 32, 64, 128, 256, 512, 1024):
        v = []
        for r in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            env.rollout(K, action_seed=7, step0=t, buffers=b)
            e1.record(stream)
            torch.cuda.synchronize()
            t += K
            if r:
                v.append(e0.elapsed_time(e1))
        ms[K] = float(np.median(v))
    Ks = np.array(list(ms), float)
    y = np.array([ms[k] for k in ms]) * 1e3
    slope, icpt = np.linalg.lstsq(np.stack([Ks, np.ones_like(Ks)], 1), y, rcond=None)[0]
    res[f"epw{epw}"] = {"kernel": kern, "bit_equal_to_epw64": bool(same),
                        "us_per_launch": {int(k): round(v * 1e3, 2) for k, v in ms.items()},
                        "fit_us_per_step": round(float(slope), 4), "fit_intercept_us": round(float(icpt), 2),
                        "env_steps_per_s_1024": N * 1024 / (ms[1024] * 1e-3)}
    print(json.dumps({f"epw{epw}": res[f"epw{epw}"]}), flush=True)
    del env, b
print(json.dumps(res))
