"""ctypes front of the parity oracle (oracle/fjsp_oracle.c).  TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / CPU baseline.  The product package never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

AGENTS = ["pickup_station", "agv", "small_machine", "big_machine",
          "packaging_blue_1", "packaging_blue_2", "packaging_red", "packaging_green"]

# status bits (mirrors FJSP_STATUS_* in include/fjsp.h)
ST_EXCEPTION = 0x1
ST_OBS_OVERFLOW = 0x2
ST_PKG_WAIT = 0x4
ST_TRAY_LOST = 0x8
ST_PROD_LOST = 0x10
ST_OVERWRITE = 0x20


class Rec(ctypes.Structure):
    _fields_ = [
        ("obs_i32", ctypes.c_int32 * 20),
        ("obs_i8", ctypes.c_int8 * 12),
        ("obs_f32", ctypes.c_float * 6),
        ("masks", ctypes.c_int8 * 29),
        ("term", ctypes.c_uint8),
        ("trunc", ctypes.c_uint8),
        ("pad", ctypes.c_uint8 * 2),
        ("rewards", ctypes.c_double * 8),
        ("sim_time", ctypes.c_double),
        ("orders_completed", ctypes.c_int32),
        ("packaged", ctypes.c_int32),
        ("results", ctypes.c_uint32 * 8),
        ("status", ctypes.c_uint32),
        ("current_step", ctypes.c_int32),
    ]


REC_DTYPE = np.dtype([
    ("obs_i32", np.int32, (20,)), ("obs_i8", np.int8, (12,)), ("obs_f32", np.float32, (6,)),
    ("masks", np.int8, (29,)), ("term", np.uint8), ("trunc", np.uint8), ("pad", np.uint8, (2,)),
    ("rewards", np.float64, (8,)), ("sim_time", np.float64), ("orders_completed", np.int32),
    ("packaged", np.int32), ("results", np.uint32, (8,)), ("status", np.uint32),
    ("current_step", np.int32)], align=True)

DEFAULT_CFG = dict(num_trays=1000, tray_capacity=5, mask_tray_capacity=5, storage_capacity=100,
                   step_size=10, max_episode_steps=200, agv_speed=1, pt_small=60, pt_big=120,
                   pt_packaging=30, packaging_capacity=20)
CFG_ORDER = ["num_trays", "tray_capacity", "mask_tray_capacity", "storage_capacity", "step_size",
             "max_episode_steps", "agv_speed", "pt_small", "pt_big", "pt_packaging",
             "packaging_capacity"]

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or (
                os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "fjsp_oracle.c"))):
            build()
        L = ctypes.CDLL(LIB_PATH)
        assert L.oracle_record_size() == ctypes.sizeof(Rec) == REC_DTYPE.itemsize
        L.oracle_create.restype = ctypes.c_void_p
        L.oracle_create.argtypes = [ctypes.POINTER(ctypes.c_int32)]
        L.oracle_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.oracle_reset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Rec)]
        L.oracle_step.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Rec)]
        L.oracle_orders.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
        L.oracle_heuristic.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_actions.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_rollout.argtypes = [ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_gae.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_void_p, ctypes.c_void_p]
        _lib = L
    return _lib


def cfg_array(**over):
    c = dict(DEFAULT_CFG)
    c.update(over)
    return (ctypes.c_int32 * len(CFG_ORDER))(*[int(c[k]) for k in CFG_ORDER])


def rec_to_np(r):
    return np.frombuffer(bytes(r), dtype=REC_DTYPE)[0]


class OracleEnv:
    """One reference-semantics env (its own MT19937 stream, like one reference process)."""

    def __init__(self, **cfg):
        self._cfg = cfg_array(**cfg)
        self._h = lib().oracle_create(self._cfg)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_destroy(self._h)
            self._h = None

    def seed(self, s):
        lib().oracle_seed(self._h, s & 0xFFFFFFFF)

    def reset(self, seed=None, num_orders=30):
        if seed is not None:
            self.seed(seed)
        r = Rec()
        lib().oracle_reset(self._h, num_orders, ctypes.byref(r))
        return rec_to_np(r)

    def step(self, actions, order=None):
        a = bytes(bytearray(int(x) & 0xFF for x in actions))
        o = None if order is None else bytes(bytearray(order))
        r = Rec()
        lib().oracle_step(self._h, a, o, ctypes.byref(r))
        return rec_to_np(r)

    def heuristic(self):
        """MultiAgentA2C._get_heuristic_actions (a2c.py:390-537) on the current state."""
        out = np.zeros(8, np.uint8)
        lib().oracle_heuristic(self._h, out.ctypes.data)
        return out

    def orders(self, max_orders=128):
        buf = (ctypes.c_uint32 * max_orders)()
        n = lib().oracle_orders(self._h, buf, max_orders)
        return np.array(buf[:min(n, max_orders)], np.uint32)


def actions(seed, env_gid, step, masks=None):
    out = np.zeros(8, np.uint8)
    m = None
    if masks is not None:
        m = np.ascontiguousarray(masks, np.int8)
    lib().oracle_actions(seed, env_gid, step, None if m is None else m.ctypes.data, out.ctypes.data)
    return out


def rollout(n_envs, steps, seeds=None, gid0=0, num_orders=30, action_seed=0, policy=0,
            actions_in=None, record=True, record_resets=False, **cfg):
    """Run n_envs envs x steps with auto-reset; returns (records [steps, n_envs], resets, checksum).
    policy: 0 unmasked random, 1 masked random, 3 heuristic (a2c.py:390-537); actions_in -> 2."""
    seeds = np.arange(gid0, gid0 + n_envs, dtype=np.uint32) if seeds is None else np.asarray(seeds, np.uint32)
    rec = np.zeros((steps, n_envs), REC_DTYPE) if record else None
    rst = np.zeros((steps, n_envs), REC_DTYPE) if record_resets else None
    ain = None
    if actions_in is not None:
        ain = np.ascontiguousarray(actions_in, np.uint8)
        policy = 2
    ck = ctypes.c_uint64(0)
    lib().oracle_rollout(cfg_array(**cfg), n_envs, gid0, seeds.ctypes.data, num_orders, steps,
                         action_seed, policy, None if ain is None else ain.ctypes.data,
                         None if rec is None else rec.ctypes.data,
                         None if rst is None else rst.ctypes.data, ctypes.byref(ck))
    return rec, rst, ck.value


def gae(rewards, values, boots, seg_end, gamma, lamb):
    """rewards f64 [T, M], values f32 [T, M], boots f64 [S, M], seg_end u8 [T]."""
    r = np.ascontiguousarray(rewards, np.float64)
    v = np.ascontiguousarray(values, np.float32)
    b = np.ascontiguousarray(boots, np.float64)
    se = np.ascontiguousarray(seg_end, np.uint8)
    T, M = r.shape
    ret = np.zeros_like(r)
    adv = np.zeros_like(r)
    for m in range(M):
        lib().oracle_gae(r[:, m:].ctypes.data, v[:, m:].ctypes.data, b[:, m:].ctypes.data,
                         se.ctypes.data, T, M, gamma, lamb, ret[:, m:].ctypes.data,
                         adv[:, m:].ctypes.data)
    return ret, adv
