"""Shared parity helpers: golden-fixture loading and exact comparisons.

The canonical per-env record matches the C-ABI SoA field order (include/fjsp.h):
obs_i32[20], obs_i8[12], obs_f32[6], masks[29], rewards f64[8], term, trunc.
"""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

BASE_CFG = {}
SCENARIO_CFG = {
    "pipeline": ({}, 5),
    "storage": ({"storage_capacity": 2}, 5),
    "overwrite": ({"tray_capacity": 3}, 5),
    "short_heur": ({"max_episode_steps": 30}, 1),
}
FIELDS = ["obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc"]


class Trace:
    def __init__(self, npz, prefix, seed, num_orders, cfg):
        self.name = prefix.rstrip("_")
        self.seed = seed
        self.num_orders = num_orders
        self.cfg = cfg
        g = lambda k: npz[prefix + k]  # noqa: E731
        self.actions = g("actions")
        self.obs_i32, self.obs_i8, self.obs_f32, self.masks = g("obs_i32"), g("obs_i8"), g("obs_f32"), g("masks")
        self.rewards, self.term, self.trunc = g("rewards"), g("term"), g("trunc")
        self.sim_time, self.orders_completed, self.packaged = g("sim_time"), g("orders_completed"), g("packaged")
        self.results = g("results")
        self.reset_i32, self.reset_i8, self.reset_f32, self.reset_masks = (
            g("reset_i32"), g("reset_i8"), g("reset_f32"), g("reset_masks"))
        self.init_i32, self.init_i8, self.init_f32, self.init_masks = (
            g("init_i32"), g("init_i8"), g("init_f32"), g("init_masks"))

    @property
    def steps(self):
        return len(self.actions)


def load_traces():
    d = np.load(os.path.join(GOLDEN, "traces.npz"))
    out = []
    for s in range(4):
        for p, n in (("unmasked", 30), ("masked", 30), ("heuristic", 2)):
            out.append(Trace(d, f"{p}_s{s}_", s, n, {}))
    return out


def load_scenarios():
    d = np.load(os.path.join(GOLDEN, "scenarios.npz"))
    out = []
    for name, (cfg, n) in SCENARIO_CFG.items():
        seeds = (3, 11) if name == "short_heur" else (0, 7)
        for s in seeds:
            out.append(Trace(d, f"{name}_s{s}_", s, n, cfg))
    return out


def load_digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


def record_bytes(obs_i32, obs_i8, obs_f32, masks, rewards, term, trunc):
    return b"".join([np.ascontiguousarray(obs_i32, np.int32).tobytes(),
                     np.ascontiguousarray(obs_i8, np.int8).tobytes(),
                     np.ascontiguousarray(obs_f32, np.float32).tobytes(),
                     np.ascontiguousarray(masks, np.int8).tobytes(),
                     np.ascontiguousarray(rewards, np.float64).tobytes(),
                     bytes([int(term), int(trunc)])])


def chunk_digests(get_record, steps, chunk):
    """get_record(t) -> tuple of per-step arrays of one env; returns hex digests per chunk."""
    row = []
    for c in range(0, steps, chunk):
        h = hashlib.sha256()
        for t in range(c, min(steps, c + chunk)):
            h.update(record_bytes(*get_record(t)))
        row.append(h.hexdigest()[:16])
    return row


def param_shapes():
    """Shapes of the learner's parameters in flat_grads order (8 stacked actors, then the critic)."""
    import importlib
    A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
    actors, critic = A.init_networks(seed=0)
    return [tuple(p.shape) for p in list(actors.parameters()) + list(critic.parameters())]


def grad_errors(got, ref):
    """Per parameter tensor (shape, ||got - ref|| / ||ref||) of two flat gradient vectors."""
    out, off = [], 0
    for shp in param_shapes():
        n = int(np.prod(shp))
        a, b = got[off:off + n].double(), ref[off:off + n].double()
        off += n
        out.append((shp, float((a - b).norm()) / max(float(b.norm()), 1e-30)))
    assert off == ref.numel() == got.numel()
    return out


def assert_grads_close(got, ref, rel=1e-5):
    """Reduced gradients vs the single learner's, per parameter tensor: ||got - ref|| <= rel *
    ||ref|| (f32 sums in another order; a missing 1/world or a double-counted shard is O(1) off)."""
    errs = grad_errors(got, ref)
    bad = [(s, e) for s, e in errs if e > rel]
    assert not bad, bad
    return errs
