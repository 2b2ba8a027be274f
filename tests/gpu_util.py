"""Helpers for the GPU parity tests: import the package and run the HIP path."""
import importlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

fjsp = importlib.import_module("multi-agent-rl-for-fjsp_amd")
vec_env = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
native = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")

CFG_KEYS = ["num_trays", "tray_capacity", "mask_tray_capacity", "storage_capacity", "step_size",
            "max_episode_steps", "agv_speed", "pt_small", "pt_big", "pt_packaging", "packaging_capacity"]


def make_env(n, **cfg):
    return vec_env.FJSPVecEnv(n, **cfg)


def to_np(b, t=None):
    """Buffers -> dict of numpy arrays with env-major layout [T, N, F]."""
    out = {}
    for k in ["obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "results", "next_i32", "next_i8",
              "next_f32", "next_masks"]:
        v = getattr(b, k, None)
        if v is not None:
            out[k] = v.transpose(1, 2).contiguous().cpu().numpy()
    for k in ["term", "trunc", "status", "orders_completed", "packaged", "sim_time"]:
        v = getattr(b, k, None)
        if v is not None:
            out[k] = v.cpu().numpy()
    if "results" in out:
        out["results"] = out["results"].view(np.uint32)
    if "status" in out:
        out["status"] = out["status"].view(np.uint32)
    return out
