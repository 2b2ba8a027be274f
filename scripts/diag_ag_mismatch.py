"""Diagnostic: first (step, env, field) where k_step_ag differs from k_step_pipe (bring-up aid)."""
import importlib, sys, os, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests import gpu_util as G

def run(agents, n, chunks, num_orders, seed, **cfg):
    env = G.make_env(n, **cfg)
    G.native.check(G.native.lib().fjsp_set_option(env.handle, b"agents", agents))
    env.reset(seeds=torch.arange(n) * int(os.environ.get("SM", "1")) + int(os.environ.get("SB", "100")), num_orders=num_orders)
    parts, t = [], 0
    for k in chunks:
        parts.append(G.to_np(env.rollout(k, action_seed=seed, step0=t, policy="random")))
        t += k
    return {key: np.concatenate([p[key] for p in parts]) for key in parts[0]}

n, chunks, no = int(os.environ.get("N", "2048")), json.loads(sys.argv[1]) if len(sys.argv) > 1 else [300, 1, 399], int(os.environ.get("NO", "1"))
seed = int(os.environ.get("AS", "5"))
a = run(1, n, chunks, no, seed)
b = run(0, n, chunks, no, seed)
first = None
for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "status"):
    d = np.argwhere(a[k] != b[k])
    if len(d):
        t = d[:, 0].min()
        e = d[d[:, 0] == t][0][1]
        print(k, "first diff step", t, "env", e, "n_diff", len(d), "envs", len(set(d[:, 1].tolist())))
        if first is None or t < first[0]:
            first = (t, e)
t, e = first
print("first", first)
for s in range(max(0, t - 3), t + 2):
    print("step", s, "term", a["term"][s, e], b["term"][s, e], "trunc", a["trunc"][s, e], b["trunc"][s, e], "status", a["status"][s, e], b["status"][s, e])
    print("  i32 ag  ", a["obs_i32"][s, e].tolist(), "\n  i32 pipe", b["obs_i32"][s, e].tolist())
    print("  i8 ag  ", a["obs_i8"][s, e].tolist(), "\n  i8 pipe", b["obs_i8"][s, e].tolist())
    print("  rew ag  ", a["rewards"][s, e].tolist(), "\n  rew pipe", b["rewards"][s, e].tolist())
    print("  f32 ag  ", a["obs_f32"][s, e].tolist(), "\n  f32 pipe", b["obs_f32"][s, e].tolist())
    print("  mask ag  ", a["masks"][s, e].tolist(), "\n  mask pipe", b["masks"][s, e].tolist())
