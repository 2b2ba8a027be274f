"""FJSPSimulation drop-in: one reference environment stepped by the HIP kernels (N = 1).

Reference: FJSPSimulation.py (class FJSPSimulation, :27-430).  Same constructor, reset(),
step(), get_order_progress(), observation_space(), action_space(), get_agent_ids() and the
attributes a2c.py reads (current_step, agv.position, agv.carrying_tray).  Observations are the
reference's dicts of numpy arrays with the exact dtypes; rewards are Python floats (fp64);
terminations / truncations are Python bools; infos carry the decoded action-result dicts.

Randomness: like the reference, reset() draws from numpy's GLOBAL legacy MT19937 stream
(np.random.seed / randint / choice, FJSPSimulation.py:107-112,298-299).  The facade hands
numpy's state to the device (fjsp_mt_set), the reset kernel draws the orders, and the advanced
state is handed back (fjsp_mt_get), so interleaving with other np.random users is identical.
"""
import ctypes

import numpy as np
import torch

from . import _native as nat
from .spec import ACTION_NAMES, AGENTS, decode_result
from .utils.ActionSpaces import ActionSpaces
from .utils.ObservationSpaces import ObservationSpaces
from .utils.RewardModel import RewardModel

# constants.py:5-32 (values of the reference configuration)
LOCATION_POSITIONS = {"PICKUP": (0, 0), "BIG_MACHINE": (0, 3), "SMALL_MACHINE": (2, 3), "STORAGE": (3, 0),
                      "PACKAGING": (3, 5)}
PROCESSING_TIMES = {"small_machine": 60, "big_machine": 120, "packaging": 30}
CONFIG = {"num_trays": 1000, "tray_capacity": 5, "num_packaging_blue": 2, "num_packaging_red": 1,
          "num_packaging_green": 1, "grid_rows": 4, "grid_cols": 6, "agv_speed": 1, "step_size": 10,
          "max_episode_steps": 200}

_AGENT_INDEX = {a: i for i, a in enumerate(AGENTS)}
_CANON = list(range(8))
_AGENT_TYPE = {"pickup_station": "PICKUP_STATION", "agv": "AGV", "small_machine": "SMALL_MACHINE",
               "big_machine": "BIG_MACHINE"}


def native_config(config):
    """The reference honours only these config keys (FJSPSimulation.py:87,92-93,183,223); the
    agents read the module CONFIG / PROCESSING_TIMES (PickupStationAgent.py:169, AGVAgent.py:390)."""
    return nat.default_config(
        num_trays=config["num_trays"], tray_capacity=config.get("tray_capacity", 5),
        mask_tray_capacity=CONFIG["tray_capacity"], storage_capacity=config.get("storage_capacity", 100),
        step_size=config["step_size"], max_episode_steps=config.get("max_episode_steps", 500),
        agv_speed=CONFIG["agv_speed"], pt_small=PROCESSING_TIMES["small_machine"],
        pt_big=PROCESSING_TIMES["big_machine"], pt_packaging=PROCESSING_TIMES["packaging"])


class _Packed:
    """All per-step outputs of one env in one pinned host record that the kernels write directly
    (zero-copy: hipHostMalloc'd memory is mapped into the GPU's address space), so a step costs one
    launch and one stream synchronisation, no copy call.  The actions are read the same way from a
    pinned 8-byte row."""
    FIELDS = [("obs_i32", np.int32, 20), ("obs_i8", np.int8, 12), ("obs_f32", np.float32, 6),
              ("masks", np.int8, 29), ("rewards", np.float64, 8), ("term", np.uint8, 1), ("trunc", np.uint8, 1),
              ("results", np.uint32, 8), ("orders_completed", np.int32, 1), ("packaged", np.int32, 1),
              ("sim_time", np.float64, 1), ("status", np.uint32, 1)]
    OBS = ("obs_i32", "obs_i8", "obs_f32", "masks", "status")

    def __init__(self):
        off = 0
        self.layout = {}
        for name, dt, n in self.FIELDS:
            off = (off + 7) & ~7
            self.layout[name] = (off, np.dtype(dt), n)
            off += np.dtype(dt).itemsize * n
        self.nbytes = (off + 7) & ~7
        self.host = torch.zeros(self.nbytes, dtype=torch.uint8).pin_memory()
        self.np = self.host.numpy()
        self.view = {name: self.np[off: off + dt.itemsize * n].view(dt) for name, (off, dt, n) in self.layout.items()}
        base = self.host.data_ptr()
        self.out_full, self.out_obs = nat.fjsp_out(), nat.fjsp_out()
        for name, (off, dt, n) in self.layout.items():
            setattr(self.out_full, name, base + off)
            if name in self.OBS:
                setattr(self.out_obs, name, base + off)
        self.ref_full, self.ref_obs = ctypes.byref(self.out_full), ctypes.byref(self.out_obs)


class _AGVView:
    """simulation.agv as a2c.py:298-305 reads it: position and carrying_tray come from the last
    observation (AGVAgent.get_observation fields position / carrying_tray / tray_product_count,
    AGVAgent.py:60-64), so reading them costs no device access."""
    def __init__(self, sim):
        self._sim = sim

    @property
    def position(self):
        o = self._sim._last_i32
        return (int(o[7]), int(o[8]))

    @property
    def carrying_tray(self):
        o = self._sim._last_i32
        return _TrayView(int(o[10])) if o[9] else None

    is_moving = False   # the AGV always arrives within the step (8 / agv_speed < step_size)


class _TrayView:
    def __init__(self, n):
        self.n_products = n

    def __len__(self):   # truthiness of a carried tray is True even when empty (reference Tray)
        return self.n_products

    def __bool__(self):
        return True


class _AgentView:
    def __init__(self, name):
        self.agent_id = name
        self.agent_type = _AGENT_TYPE.get(name, "PACKAGING")

    def get_observation_space(self):
        if self.agent_id == "pickup_station":
            return ObservationSpaces.pickup_station()
        if self.agent_id == "agv":
            return ObservationSpaces.agv()
        if self.agent_id in ("small_machine", "big_machine"):
            return getattr(ObservationSpaces, self.agent_id)()
        return ObservationSpaces.packaging()

    def get_action_space(self):
        if self.agent_id.startswith("packaging"):
            return ActionSpaces.packaging()
        return getattr(ActionSpaces, self.agent_id)()


def _action_code(v):
    """Reference branch semantics by value: 0..max valid, anything else behaves as invalid."""
    try:
        if isinstance(v, torch.Tensor):
            v = v.item()
        if isinstance(v, (float, np.floating)):
            if float(v).is_integer():
                v = int(v)
            else:
                return 254
        v = int(v)
    except (TypeError, ValueError):
        return 254
    return v if 0 <= v <= 253 else 254


class FJSPSimulation:
    """One reference environment on the GPU (drop-in for FJSPSimulation.py:27)."""

    def __init__(self, config=None, device=None):
        if not torch.cuda.is_available():
            raise nat.FjspNativeError("FJSPSimulation needs a GPU (HIP); there is no CPU fallback")
        from .vec_env import FJSPVecEnv
        self.config = config or CONFIG
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._venv = FJSPVecEnv(1, device=self.device, config=native_config(self.config))
        self._h = self._venv.handle
        self._L = nat.lib()
        # the observation dicts built in C (csrc/fjsp_facade.c; spec.obs_dicts is its definition),
        # and the common step (a canonical dict of plain ints on the step server) in one C call
        F = nat.facade()
        self._obs_dicts = F.obs_dicts
        self._fast_step = F.step
        self._stepper = None
        # one launch per step: no per-launch event pair (fjsp_last_kernel_ms), the facade never reads it
        nat.check(self._L.fjsp_set_option(self._h, b"timing", 0))
        self._packed = _Packed()
        self._act_host = torch.zeros(8, dtype=torch.uint8).pin_memory()   # read by the kernel in place
        self._act_np = self._act_host.numpy()
        self._act_ptr = ctypes.c_void_p(self._act_host.data_ptr())
        self._stream = None
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.reward_calculator = RewardModel()
        self._pushed_weights = None
        self._pushed_rc = None
        self.agents = {a: _AgentView(a) for a in AGENTS}
        self.agv = _AGVView(self)
        self.current_step = 0
        self.total_products_packaged = 0
        self.sim_time = 0
        self._orders_total = 0
        self._last_obs = None
        self._viewcache = None
        self._infocache = {}
        # the step server (fjsp_server_*): a resident kernel stepping this env on a host doorbell;
        # configured at the first canonical-order step, relaunched by the library after any other
        # call on the handle (reset, read_env, a reward-weight upload, a non-canonical step)
        self.use_server = True
        self._srv_on = False
        # an empty episode (no orders, no RNG draws), like a freshly constructed reference sim
        self._bind_stream()
        nat.check(self._L.fjsp_reset(self._h, None, None, 0, self._packed.ref_obs))
        self._wait()
        self._take_obs(self._packed.view)

    # ------------------------------------------------------------------ internals
    def _bind_stream(self):
        """Launch on torch's current stream of the device (re-read every call, as vec_env does;
        the raw handle query is the cheap form of torch.cuda.current_stream(device).cuda_stream)."""
        s = torch._C._cuda_getCurrentRawStream(self._dev_index)
        if s != self._stream:
            nat.check(self._L.fjsp_set_stream(self._h, ctypes.c_void_p(s)))
            self._stream = s

    def _wait(self):
        nat.check(self._L.fjsp_sync(self._h))

    def _view(self):
        if self._viewcache is None:
            self._viewcache = self._venv.read_env(0)
        return self._viewcache

    def _push_weights(self):
        """The kernel's reward table follows reward_calculator's weights (read before every step,
        like the reference's step reads them); re-uploaded only when an attribute changed."""
        rc = self.reward_calculator
        d = vars(rc)
        if rc is self._pushed_rc and d == self._pushed_weights:
            return
        w = rc.weights()
        rw = nat.fjsp_reward_weights(*w)
        nat.check(self._L.fjsp_set_reward_weights(self._h, ctypes.byref(rw)))
        self._pushed_rc, self._pushed_weights = rc, dict(d)

    def _take_obs(self, p):
        self._last_i32 = p["obs_i32"]   # the record's view: the AGV reads see the latest observation
        self._last_obs = self._obs_dicts(p["obs_i32"], p["obs_i8"], p["obs_f32"], p["masks"])
        return self._last_obs

    def _info(self, i, a, act, word):
        key = (i, act, word)
        d = self._infocache.get(key)
        if d is None:
            d = self._infocache[key] = decode_result(a, act, word)
        return dict(d)

    # ------------------------------------------------------------------ reference API
    def reset(self, seed=None, num_orders=None):
        """FJSPSimulation.reset (FJSPSimulation.py:286-323)."""
        if seed is not None:
            np.random.seed(seed)
        n = num_orders if num_orders is not None else 30
        st = np.random.get_state()
        self._bind_stream()
        self._venv.mt_set(0, np.asarray(st[1], np.uint32), int(st[2]))
        nat.check(self._L.fjsp_reset(self._h, None, None, int(n), self._packed.ref_obs))
        key, pos = self._venv.mt_get(0)   # synchronises the stream
        np.random.set_state((st[0], key, pos, st[3], st[4]))
        self.current_step = 0
        self.total_products_packaged = 0
        self.sim_time = 0
        self._orders_total = int(n)
        self._viewcache = None
        obs = self._take_obs(self._packed.view)
        return obs, {a: {} for a in AGENTS}

    def _make_stepper(self):
        P = self._packed
        fn = ctypes.cast(self._L.fjsp_server_step_actions, ctypes.c_void_p).value
        offs = [P.layout[k][0] for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc",
                                         "results", "orders_completed", "packaged", "sim_time")]
        return nat.facade().stepper(self._h.value, fn, self._act_host.data_ptr(), P.host.data_ptr(), offs,
                                    decode_result)

    def step(self, actions):
        """FJSPSimulation.step (FJSPSimulation.py:144-242)."""
        if self._srv_on and self.use_server:
            # the common case in C (_facade.step: the eight agents in dict order, plain int actions);
            # anything else returns None untouched and takes the path below
            self._push_weights()
            self._bind_stream()
            r = self._fast_step(self._stepper, actions)
            if r is not None:
                if type(r) is int:
                    nat.check(r)
                obs, rewards, terms, truncs, infos, self.sim_time, self.total_products_packaged = r
                self._last_obs = obs
                self._viewcache = None
                self.current_step += 1
                return obs, rewards, terms, truncs, infos
        codes = self._act_np
        codes.fill(255)   # an agent absent from the dict does not act
        order = []
        for k, v in actions.items():
            i = _AGENT_INDEX.get(k)
            if i is None or i in order:
                continue
            codes[i] = v if (type(v) is int and 0 <= v <= 253) else _action_code(v)
            order.append(i)
        canon = order == _CANON
        ord_arr = None
        if not canon:
            order += [i for i in range(8) if i not in order]
            canon = order == _CANON
            ord_arr = None if canon else (ctypes.c_uint8 * 8)(*order)
        self._push_weights()
        self._bind_stream()
        if canon and self.use_server:
            if not self._srv_on:   # inline mode: the 8 action bytes ride in the doorbell's cache line
                nat.check(self._L.fjsp_server_start(self._h, None, 0, self._packed.ref_full))
                self._stepper = self._make_stepper()
                self._srv_on = True
            nat.check(self._L.fjsp_server_step_actions(self._h, self._act_ptr))   # returns with the record written
        else:
            nat.check(self._L.fjsp_step(self._h, self._act_ptr, ord_arr, 0, self._packed.ref_full))
            self._wait()
        p = self._packed.view   # every value leaves the pinned record as Python numbers or fresh arrays
        self._viewcache = None
        obs = self._take_obs(p)
        rw = p["rewards"].tolist()
        rewards = dict(zip(AGENTS, rw))
        term = bool(p["term"][0])
        trunc = bool(p["trunc"][0])
        self.sim_time = float(p["sim_time"][0])
        self.total_products_packaged = int(p["packaged"][0])
        oc = int(p["orders_completed"][0])
        res = p["results"].tolist()
        infos = {}
        for i, a in enumerate(AGENTS):
            act = actions.get(a, 0)
            d = self._info(i, a, act, res[i]) if type(act) is int else decode_result(a, act, res[i])
            d_all = {"action_result": d, "sim_time": self.sim_time, "orders_completed": oc,
                     "total_products_packaged": self.total_products_packaged}
            infos[a] = d_all
        self.current_step += 1
        return obs, rewards, {a: term for a in AGENTS}, {a: trunc for a in AGENTS}, infos

    def get_observations(self):
        return self._last_obs

    def get_order_progress(self):
        """FJSPSimulation.get_order_progress (FJSPSimulation.py:260-284)."""
        v = self._view()
        detail = []
        for i in range(v.num_orders):
            w = int(v.orders[i])
            detail.append({"order_id": i, "total_products": w & 15, "processed": (w >> 8) & 15,
                           "packaged": (w >> 12) & 15, "is_complete": bool((w >> 16) & 1)})
        return {"total_orders": v.num_orders, "completed_orders": v.orders_completed,
                "total_products": sum(d["total_products"] for d in detail),
                "products_processed": sum(d["processed"] for d in detail),
                "products_packaged": v.total_packaged, "orders_detail": detail}

    def get_agent_ids(self):
        return list(AGENTS)

    def observation_space(self, agent_id):
        return self.agents[agent_id].get_observation_space()

    def action_space(self, agent_id):
        return self.agents[agent_id].get_action_space()

    def _get_action_names(self, actions):
        return {a: (ACTION_NAMES[a][v] if a in ACTION_NAMES and 0 <= v < len(ACTION_NAMES[a]) else f"ACTION_{v}")
                for a, v in actions.items()}

    @property
    def orders_count(self):
        return self._orders_total
