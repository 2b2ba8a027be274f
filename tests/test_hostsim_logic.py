"""CPU check of the kernel's closed-form state machine (csrc/fjsp_env.h compiled for the host
by tests/hostsim, TEST-ONLY) against the oracle's event-heap restatement and the reference's
golden traces.  The GPU tests (test_gpu_parity.py) are the parity proof of the HIP path; this
keeps the shared step logic covered in the CPU-only CI."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from tests import parity_util as P

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "hostsim", "libhostsim.so")
SRC = [os.path.join(HERE, "hostsim", "hostsim.cpp"),
       os.path.join(os.path.dirname(HERE), "multi-agent-rl-for-fjsp_amd", "csrc", "fjsp_env.h")]


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(SO) or any(os.path.getmtime(s) > os.path.getmtime(SO) for s in SRC):
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wno-unknown-pragmas",
                        "-o", SO, SRC[0]], check=True)
    lib = ctypes.CDLL(SO)
    Pt = ctypes.c_void_p
    lib.hs_create.restype = Pt
    lib.hs_create.argtypes = [Pt, ctypes.c_int]
    lib.hs_destroy.argtypes = [Pt]
    lib.hs_reset.argtypes = [Pt, Pt, ctypes.c_int, Pt, Pt, Pt, Pt]
    lib.hs_step.argtypes = [Pt, Pt, ctypes.c_int] + [Pt] * 13
    lib.hs_heuristic.argtypes = [Pt, Pt]
    return lib


class HS:
    def __init__(self, L, n, cfg):
        self.L, self.n = L, n
        self.h = L.hs_create(O.cfg_array(**cfg), n)
        z = np.zeros
        self.i32, self.i8, self.f32, self.mk = z((n, 20), np.int32), z((n, 12), np.int8), z((n, 6), np.float32), z((n, 29), np.int8)
        self.rew, self.term, self.trunc = z((n, 8)), z(n, np.uint8), z(n, np.uint8)
        self.res, self.st = z((n, 8), np.uint32), z(n, np.uint32)
        self.ri32, self.ri8, self.rf32, self.rmk = (np.zeros_like(self.i32), np.zeros_like(self.i8),
                                                    np.zeros_like(self.f32), np.zeros_like(self.mk))

    def __del__(self):
        self.L.hs_destroy(self.h)

    def heuristic(self):
        out = np.zeros((self.n, 8), np.uint8)
        self.L.hs_heuristic(self.h, out.ctypes.data)
        return out

    def reset(self, seeds, num_orders):
        s = np.ascontiguousarray(seeds, np.uint32)
        self.L.hs_reset(self.h, s.ctypes.data, num_orders, self.i32.ctypes.data, self.i8.ctypes.data,
                        self.f32.ctypes.data, self.mk.ctypes.data)

    def step(self, acts):
        a = np.ascontiguousarray(acts, np.uint8)
        self.L.hs_step(self.h, a.ctypes.data, 1, *[x.ctypes.data for x in (
            self.i32, self.i8, self.f32, self.mk, self.rew, self.term, self.trunc, self.res, self.st,
            self.ri32, self.ri8, self.rf32, self.rmk)])


@pytest.mark.parametrize("policy,cfg,norders,n,steps", [
    (0, {}, 30, 64, 1000),
    (1, {}, 30, 64, 1000),
    (0, {"storage_capacity": 2}, 5, 32, 500),
    (1, {"tray_capacity": 3, "max_episode_steps": 50}, 3, 32, 500),
    (1, {"packaging_capacity": 2, "num_trays": 40}, 20, 32, 600),
])
def test_closed_form_vs_oracle(L, policy, cfg, norders, n, steps):
    hs = HS(L, n, cfg)
    seeds = np.arange(n, dtype=np.uint32) + 100
    hs.reset(seeds, norders)
    rec, rst, _ = O.rollout(n, steps, seeds=seeds, gid0=0, num_orders=norders, policy=policy,
                            record_resets=True, **cfg)
    masks = hs.mk.copy()
    for t in range(steps):
        acts = np.stack([O.actions(0, e, t, masks[e] if policy == 1 else None) for e in range(n)])
        hs.step(acts)
        R = rec[t]
        # the kernel flags (and stops emulating) paths the oracle emulates by the event heap:
        # a packaging Request that waits (users == capacity) or the reference raising
        k_div = (hs.st & 1) != 0
        o_div = (R["status"] & (O.ST_EXCEPTION | O.ST_PKG_WAIT | O.ST_OBS_OVERFLOW)) != 0
        assert np.array_equal(k_div, o_div), t
        ok_env = ~k_div
        for name, mine in (("obs_i32", hs.i32), ("obs_i8", hs.i8), ("obs_f32", hs.f32), ("masks", hs.mk),
                           ("rewards", hs.rew), ("term", hs.term), ("trunc", hs.trunc), ("results", hs.res)):
            a, b = mine[ok_env], np.asarray(R[name])[ok_env]
            assert a.tobytes() == np.ascontiguousarray(b).tobytes(), (t, name)
        masks = hs.rmk.copy()


@pytest.mark.parametrize("tr", P.load_traces() + P.load_scenarios(), ids=lambda t: t.name)
def test_closed_form_vs_golden(L, tr):
    hs = HS(L, 1, tr.cfg)
    hs.reset([tr.seed], tr.num_orders)
    assert P.bits_equal(hs.i32[0], tr.init_i32)
    for t in range(tr.steps):
        hs.step(tr.actions[t:t + 1])
        for name, mine in (("obs_i32", hs.i32), ("obs_i8", hs.i8), ("obs_f32", hs.f32), ("masks", hs.mk),
                           ("rewards", hs.rew), ("results", hs.res)):
            assert P.bits_equal(mine[0], getattr(tr, name)[t]), (tr.name, t, name)
        assert P.bits_equal(hs.ri32[0], tr.reset_i32[t]), (tr.name, t)


def test_heuristic_vs_golden_probe(L):
    """heuristic_actions (the kernel's FJSP_ACTIONS_HEURISTIC) == a2c._get_heuristic_actions on
    every pre-step state of the reference's mixed heuristic/random rollouts."""
    d = np.load(f"{P.GOLDEN}/heur_probe.npz")
    for seed in range(6):
        acts, heur = d[f"s{seed}_actions"], d[f"s{seed}_heur"]
        hs = HS(L, 1, {})
        hs.reset([seed], 30)
        for t in range(len(acts)):
            assert hs.heuristic()[0].tolist() == heur[t].tolist(), (seed, t)
            hs.step(acts[t:t + 1])


def test_heuristic_vs_oracle_rollout(L):
    """Closed-loop heuristic rollouts (policy 3): kernel logic and oracle agree step by step."""
    n, steps, norders = 32, 600, 4
    hs = HS(L, n, {})
    seeds = np.arange(n, dtype=np.uint32) + 7
    hs.reset(seeds, norders)
    rec, _, _ = O.rollout(n, steps, seeds=seeds, num_orders=norders, policy=3)
    done = 0
    for t in range(steps):
        hs.step(hs.heuristic())
        for name, mine in (("obs_i32", hs.i32), ("masks", hs.mk), ("rewards", hs.rew), ("term", hs.term)):
            assert mine.tobytes() == np.ascontiguousarray(rec[t][name]).tobytes(), (t, name)
        done += int(hs.term.sum())
    assert done > 0   # the heuristic finishes small episodes


def test_property_random_configs_and_actions(L):
    """Property test (hypothesis): the kernel's state machine equals the oracle's event heap on
    random valid configurations and arbitrary action streams, including out-of-range actions."""
    hyp = pytest.importorskip("hypothesis")
    st = hyp.strategies

    @hyp.settings(max_examples=25, deadline=None, derandomize=True)
    @hyp.given(seed=st.integers(0, 2**31 - 1), norders=st.integers(0, 12),
               tray_cap=st.integers(1, 7), storage=st.integers(0, 6), trays=st.integers(1, 60),
               step=st.sampled_from([10, 20]), acts=st.lists(st.lists(st.integers(0, 9), min_size=8, max_size=8),
                                                             min_size=40, max_size=120))
    def run(seed, norders, tray_cap, storage, trays, step, acts):
        cfg = {"tray_capacity": tray_cap, "mask_tray_capacity": tray_cap, "storage_capacity": storage,
               "num_trays": trays, "step_size": step, "pt_small": 6 * step, "pt_big": 12 * step,
               "pt_packaging": 3 * step}
        hs = HS(L, 1, cfg)
        hs.reset([seed], norders)
        o = O.OracleEnv(**cfg)
        o.reset(seed=seed, num_orders=norders)
        for a in acts:
            a = np.array(a, np.uint8)
            hs.step(a[None])
            r = o.step(a)
            if r["status"] & (O.ST_EXCEPTION | O.ST_PKG_WAIT | O.ST_OBS_OVERFLOW):
                break
            for name, mine in (("obs_i32", hs.i32), ("obs_i8", hs.i8), ("masks", hs.mk), ("rewards", hs.rew),
                               ("results", hs.res)):
                assert np.ascontiguousarray(mine[0]).tobytes() == np.ascontiguousarray(r[name]).tobytes(), name
            if r["term"] or r["trunc"]:
                o.reset(num_orders=norders)
    run()
