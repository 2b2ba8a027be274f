"""Soak: k_step_ag against k_step_pipe on larger and varied
workloads than the unit tests: every lean output compared bit for bit, launch after launch.
Prints one JSON line per case; exit status 1 on any mismatch."""
import importlib, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tests import gpu_util as G

LEAN = ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "status")
CASES = [
    dict(n=16384, orders=30, chunks=[1000, 1000, 7], cfg={}),
    dict(n=4096, orders=1, chunks=[500, 333, 1000], cfg={}),
    dict(n=2048, orders=64, chunks=[999, 1001], cfg=dict(tray_capacity=2, mask_tray_capacity=2)),
    dict(n=3000, orders=8, chunks=[700, 700], cfg=dict(storage_capacity=2, packaging_capacity=3, max_episode_steps=60)),
    dict(n=8192, orders=12, chunks=[1000, 1000], cfg=dict(pt_small=10, pt_big=20, pt_packaging=10)),
]
bad = 0
for i, c in enumerate(CASES):
    runs = []
    for agents in (1, 0):
        env = G.make_env(c["n"], **c["cfg"])
        lib = G.native.lib()
        G.native.check(lib.fjsp_set_option(env.handle, b"agents", agents))
        env.reset(seeds=torch.arange(c["n"]) * 7 + i, num_orders=c["orders"])
        out, t = {k: [] for k in LEAN}, 0
        for k in c["chunks"]:
            b = G.to_np(env.rollout(k, action_seed=100 + i, step0=t, policy="random"))
            t += k
            for key in LEAN:
                out[key].append(b[key])
        runs.append(({k: np.concatenate(v) for k, v in out.items()}, env.last_kernel()))
        del env
    ref = runs[-1][0]
    diffs = {name: [k for k in LEAN if not np.array_equal(r[k].view(np.uint8), ref[k].view(np.uint8))] for r, name in runs[:-1]}
    ends = int((ref["term"] | ref["trunc"]).sum())
    ok = all(not d for d in diffs.values())
    bad += not ok
    print(json.dumps({"case": i, "n": c["n"], "num_orders": c["orders"], "steps": sum(c["chunks"]), "cfg": c["cfg"],
                      "episode_ends": ends, "mismatching_fields": diffs, "ok": ok}), flush=True)
sys.exit(1 if bad else 0)
