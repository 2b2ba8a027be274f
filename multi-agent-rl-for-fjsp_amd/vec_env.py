"""FJSPVecEnv — N reference environments stepped in lockstep on one MI355X.

Device-resident tensors in, device-resident tensors out (zero copy through the C-ABI).
All layouts are field-major SoA with the env index fastest ([F, N]), the layout the
kernels write coalesced; ``.t()`` gives the [N, F] view a network consumes.
"""
import ctypes

import numpy as np
import torch

from . import _native as nat
from .spec import AGENTS

NI32, NI8, NF32, NMASK, NA, NFEAT = 20, 12, 6, 29, 8, 38
POLICIES = {"random": 0, "unmasked": 0, "masked": 1, "heuristic": 2}   # FJSP_ACTIONS_*


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class Buffers:
    """Output tensors for T steps of N envs (T = 1 for step/reset)."""

    def __init__(self, T, N, device, infos=True, next_obs=False, feats=False, obs=True):
        z = lambda *s, dt: torch.zeros(*s, dtype=dt, device=device)  # noqa: E731
        # feats: a2c global-state features f32 [T, 38, N] of the post-auto-reset observation
        self.feats = z(T, NFEAT, N, dt=torch.float32) if feats else None
        if not obs:   # a2c-only outputs: features, post-reset masks, rewards, term, trunc
            self.obs_i32 = self.obs_i8 = self.obs_f32 = self.masks = None
            self.results = self.orders_completed = self.packaged = self.sim_time = None
            self.next_i32 = self.next_i8 = self.next_f32 = None
            self.next_masks = z(T, NMASK, N, dt=torch.int8)
            self.rewards = z(T, NA, N, dt=torch.float64)
            self.term = z(T, N, dt=torch.uint8)
            self.trunc = z(T, N, dt=torch.uint8)
            self.status = z(T, N, dt=torch.int32)
            return
        self.obs_i32 = z(T, NI32, N, dt=torch.int32)
        self.obs_i8 = z(T, NI8, N, dt=torch.int8)
        self.obs_f32 = z(T, NF32, N, dt=torch.float32)
        self.masks = z(T, NMASK, N, dt=torch.int8)
        self.rewards = z(T, NA, N, dt=torch.float64)
        self.term = z(T, N, dt=torch.uint8)
        self.trunc = z(T, N, dt=torch.uint8)
        self.status = z(T, N, dt=torch.int32)
        if infos:
            self.results = z(T, NA, N, dt=torch.int32)
            self.orders_completed = z(T, N, dt=torch.int32)
            self.packaged = z(T, N, dt=torch.int32)
            self.sim_time = z(T, N, dt=torch.float64)
        else:
            self.results = self.orders_completed = self.packaged = self.sim_time = None
        if next_obs:
            self.next_i32 = z(T, NI32, N, dt=torch.int32)
            self.next_i8 = z(T, NI8, N, dt=torch.int8)
            self.next_f32 = z(T, NF32, N, dt=torch.float32)
            self.next_masks = z(T, NMASK, N, dt=torch.int8)
        else:
            self.next_i32 = self.next_i8 = self.next_f32 = self.next_masks = None

    def struct(self):
        o = nat.fjsp_out()
        for k in nat.OUT_FIELDS:
            t = getattr(self, k, None)
            setattr(o, k, t.data_ptr() if t is not None else None)
        return o


class FJSPVecEnv:
    """N independent FJSP environments (reference semantics per env) on one GPU.

    Env ``e`` has global id ``env_id_base + e``; its default MT19937 stream is
    ``np.random.seed(global id)`` and synthetic actions are keyed by the global id, so
    results do not depend on how envs are sharded over GPUs.
    """

    def __init__(self, num_envs, device=None, config=None, env_id_base=0, **cfg_over):
        if not torch.cuda.is_available():
            raise nat.FjspNativeError("FJSPVecEnv needs a GPU (HIP); no CPU fallback exists")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.num_envs = int(num_envs)
        self.env_id_base = int(env_id_base)
        c = config if config is not None else nat.default_config(**cfg_over)
        self.config = c
        L = nat.lib()
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            nat.check(L.fjsp_create(ctypes.byref(c), self.num_envs, self.device.index or 0,
                                    ctypes.c_void_p(stream), ctypes.byref(h)))
        self._h = h
        self._step_buf = None
        self._num_orders = 30
        self._pending_seeds = None
        if self.env_id_base:
            # default streams keyed by global id: env e starts from np.random.seed(env_id_base + e),
            # whichever call resets it first (reset(seed=None), a learner's reset, ...)
            nat.check(L.fjsp_set_option(h, b"env_id_base", self.env_id_base))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                nat.lib().fjsp_destroy(h)
            except Exception:
                pass
            self._h = None

    # ------------------------------------------------------------------ helpers
    def _sync_stream(self):
        nat.check(nat.lib().fjsp_set_stream(self._h, ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))

    @property
    def handle(self):
        return self._h

    def state_bytes_per_env(self):
        return int(nat.lib().fjsp_state_bytes(self._h))

    def seed(self, seeds):
        """np.random.seed(seeds[e]) for every env (applied at the next reset)."""
        self._pending_seeds = torch.as_tensor(seeds, device=self.device).to(torch.int64).bitwise_and(0xFFFFFFFF).to(torch.int32)

    # ------------------------------------------------------------------ API
    def reset(self, seeds=None, env_mask=None, num_orders=30, buffers=None):
        """FJSPSimulation.reset for the selected envs (FJSPSimulation.py:286-323)."""
        self._sync_stream()
        self._num_orders = int(num_orders)
        if seeds is None and getattr(self, "_pending_seeds", None) is not None:
            seeds = self._pending_seeds
        self._pending_seeds = None
        s = None
        if seeds is not None:
            s = torch.as_tensor(seeds, device=self.device)
            s = s.to(torch.int64).bitwise_and(0xFFFFFFFF).to(torch.int32).contiguous()
        m = None
        if env_mask is not None:
            m = torch.as_tensor(env_mask, device=self.device).to(torch.uint8).contiguous()
        b = buffers or Buffers(1, self.num_envs, self.device, infos=False)
        out = b.struct()
        nat.check(nat.lib().fjsp_reset(self._h, _ptr(s), _ptr(m), self._num_orders, ctypes.byref(out)))
        return b

    def step(self, actions, agent_order=None, autoreset=True, buffers=None):
        """One FJSPSimulation.step per env (FJSPSimulation.py:144-242).

        actions: uint8 tensor [8, N] (agent-major) on the env's device."""
        self._sync_stream()
        a = actions
        if a.dtype != torch.uint8 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.uint8).contiguous()
        if tuple(a.shape) != (NA, self.num_envs):
            raise ValueError(f"actions must be [8, {self.num_envs}], got {tuple(a.shape)}")
        if buffers is None:
            if self._step_buf is None:
                self._step_buf = Buffers(1, self.num_envs, self.device, infos=True, next_obs=True)
            buffers = self._step_buf
        order = None
        if agent_order is not None:
            order = (ctypes.c_uint8 * 8)(*[int(x) for x in agent_order])
        out = buffers.struct()
        nat.check(nat.lib().fjsp_step(self._h, _ptr(a), order, int(bool(autoreset)), ctypes.byref(out)))
        return buffers

    def server_start(self, actions, autoreset=True, buffers=None):
        """Start the step server (fjsp_server_start): a resident kernel that steps every env once
        per server_step() on a host doorbell, no launch or stream synchronisation per step.
        actions: u8 [8, N] the caller rewrites before every server_step (pinned host memory, or a
        device tensor whose writes are complete); outputs go to `buffers` (T = 1).  actions=None on
        a one-env handle: inline mode, each server_step(actions) hands its 8 action bytes over in
        the doorbell's cache line (fjsp_server_step_actions)."""
        if actions is None:
            if self.num_envs != 1:
                raise ValueError("inline actions (actions=None) need a one-env handle")
        else:
            if actions.dtype != torch.uint8 or not actions.is_contiguous() or tuple(actions.shape) != (NA, self.num_envs):
                raise ValueError(f"actions must be a contiguous uint8 [8, {self.num_envs}] tensor")
            if actions.device.type == "cpu" and not actions.is_pinned():
                raise ValueError("host actions must be in pinned memory (the kernel reads them in place)")
        self._srv_inline = actions is None
        self._sync_stream()
        b = buffers or Buffers(1, self.num_envs, self.device, infos=False)
        self._srv_keep = (actions, b, b.struct())          # the kernel reads / writes these every step
        nat.check(nat.lib().fjsp_server_start(self._h, _ptr(actions), int(bool(autoreset)),
                                              ctypes.byref(self._srv_keep[2])))
        return b

    def server_step(self, actions=None):
        """One step of every env on the running (or relaunched) step server; returns when the
        step's outputs are written.  Inline mode: actions = the env's 8 action codes."""
        if getattr(self, "_srv_inline", False):
            a = np.ascontiguousarray(actions, dtype=np.uint8).reshape(-1)
            if a.size != NA:
                raise ValueError("inline server_step takes the env's 8 action codes")
            nat.check(nat.lib().fjsp_server_step_actions(self._h, ctypes.c_void_p(a.ctypes.data)))
        else:
            nat.check(nat.lib().fjsp_server_step(self._h))

    def server_stop(self):
        nat.check(nat.lib().fjsp_server_stop(self._h))

    def rollout(self, K, action_seed=0, step0=0, masked=False, autoreset=True, buffers=None, infos=False,
                policy=None):
        """K fused steps with on-device actions; returns [K, F, N] trajectories.

        policy: "random" (uniform, action_space.sample()), "masked" (uniform over valid
        actions) or "heuristic" (MultiAgentA2C._get_heuristic_actions, a2c.py:390-537)."""
        self._sync_stream()
        mode = POLICIES[policy] if policy is not None else (1 if masked else 0)
        b = buffers or Buffers(K, self.num_envs, self.device, infos=infos)
        out = b.struct()
        nat.check(nat.lib().fjsp_step_many(self._h, int(K), int(action_seed) & (2**64 - 1), self.env_id_base,
                                           int(step0), mode, int(bool(autoreset)), ctypes.byref(out)))
        return b

    def evaluate(self, policy="heuristic", num_orders=5, max_steps=500, seeds=None, action_seed=0):
        """MultiAgentA2C.test (a2c.py:539-645) for every env at once: each env runs from a reset
        until its episode ends (term or trunc: the reference's `while env.agents`) or max_steps.
        Returns the reference's test() dict with one entry per env: steps, orders_completed,
        products_packaged, rewards_by_agent [8, N] (each agent's rewards summed in step order,
        as episode_rewards) and total_reward (their sum in agent order, a2c.py:626)."""
        import numpy as np
        self.reset(seeds=seeds, num_orders=num_orders)
        b = self.rollout(int(max_steps), action_seed=action_seed, policy=policy, autoreset=False, infos=True)
        done = (b.term | b.trunc).cpu().numpy().astype(bool)                  # [T, N]
        T = done.shape[0]
        first = np.where(done.any(0), done.argmax(0) + 1, T)                  # steps run per env
        live = np.arange(T)[:, None] < first[None, :]
        rew = np.where(live[:, None, :], b.rewards.cpu().numpy(), 0.0)        # [T, 8, N]
        by_agent = np.cumsum(rew, axis=0)[-1] if T else np.zeros((NA, self.num_envs))   # sequential
        idx = np.maximum(first - 1, 0)
        cols = np.arange(self.num_envs)
        pick = lambda x: x.cpu().numpy()[idx, cols] if T else np.zeros(self.num_envs, np.int32)  # noqa: E731
        return {"steps": first, "orders_completed": pick(b.orders_completed),
                "products_packaged": pick(b.packaged), "total_orders": num_orders,
                "rewards_by_agent": by_agent, "total_reward": np.cumsum(by_agent, axis=0)[-1]}

    def pack_a2c(self, feats=None, masks=None):
        """a2c features f32 [38, N] and masks int8 [29, N] of the current observations
        (MultiAgentA2C._get_global_state, a2c.py:153-166)."""
        self._sync_stream()
        if feats is None:
            feats = torch.empty(NFEAT, self.num_envs, dtype=torch.float32, device=self.device)
        if masks is None:
            masks = torch.empty(NMASK, self.num_envs, dtype=torch.int8, device=self.device)
        nat.check(nat.lib().fjsp_pack_a2c(self._h, _ptr(feats), _ptr(masks)))
        return feats, masks

    def snapshot(self, out=None):
        """Copy of every env's complete state (uint8 tensor; device unless `out` is given)."""
        self._sync_stream()
        nb = int(nat.lib().fjsp_snapshot_bytes(self._h))
        if out is None:
            out = torch.empty(nb, dtype=torch.uint8, device=self.device)
        if out.numel() * out.element_size() != nb:
            raise ValueError(f"snapshot needs {nb} bytes")
        nat.check(nat.lib().fjsp_snapshot(self._h, _ptr(out)))
        return out

    def restore(self, snap):
        self._sync_stream()
        nb = int(nat.lib().fjsp_snapshot_bytes(self._h))
        if snap.numel() * snap.element_size() != nb:
            raise ValueError(f"snapshot of {snap.numel() * snap.element_size()} bytes, handle needs {nb}")
        nat.check(nat.lib().fjsp_restore(self._h, _ptr(snap.contiguous())))

    def last_kernel(self):
        """Name of the kernel variant of the last step launch (e.g. "k_step_pipe<lds>")."""
        return nat.lib().fjsp_last_kernel(self._h).decode()

    def last_kernel_ms(self):
        ms = ctypes.c_float()
        nat.check(nat.lib().fjsp_last_kernel_ms(self._h, ctypes.byref(ms)))
        return ms.value

    def read_env(self, e):
        v = nat.fjsp_env_view()
        nat.check(nat.lib().fjsp_read_env(self._h, int(e), ctypes.byref(v)))
        return v

    def mt_get(self, e):
        import numpy as np
        key = np.zeros(624, np.uint32)
        pos = ctypes.c_int32()
        nat.check(nat.lib().fjsp_mt_get(self._h, int(e), ctypes.c_void_p(key.ctypes.data), ctypes.byref(pos)))
        return key, pos.value

    def mt_set(self, e, key, pos):
        import numpy as np
        k = np.ascontiguousarray(key, dtype=np.uint32)
        nat.check(nat.lib().fjsp_mt_set(self._h, int(e), ctypes.c_void_p(k.ctypes.data), int(pos)))

    def sync(self):
        nat.check(nat.lib().fjsp_sync(self._h))

    def faults(self, clear=False):
        """The handle's fault word (fjsp_faults; synchronises): bit 0 = a bounded hand-off wait
        of a multi-wave step kernel gave up (its envs carry FJSP_STATUS_SPIN_TIMEOUT)."""
        w = ctypes.c_uint32()
        nat.check(nat.lib().fjsp_faults(self._h, ctypes.byref(w), int(bool(clear))))
        return w.value


def gae(rewards, values, done, boot, gamma, lamb, out_ret=None, out_adv=None):
    """Returns + GAE (transition_memory.py:83-105) on device tensors.

    rewards f64 [T, M], values f32 or f64 [T, M], done u8 [T, N], boot f64 [M]; columns m = a*N + e."""
    T, M = rewards.shape
    N = done.shape[1]
    ret = out_ret if out_ret is not None else torch.empty_like(rewards)
    adv = out_adv if out_adv is not None else torch.empty_like(rewards)
    r = rewards.contiguous(); v = values.contiguous(); d = done.to(torch.uint8).contiguous(); b = boot.contiguous()
    stream = torch.cuda.current_stream(rewards.device).cuda_stream
    fn = nat.lib().fjsp_gae_f64 if v.dtype == torch.float64 else nat.lib().fjsp_gae
    if v.dtype not in (torch.float32, torch.float64):
        raise TypeError("values must be float32 or float64")
    nat.check(fn(_ptr(r), _ptr(v), _ptr(d), _ptr(b), T, N, M, float(gamma), float(lamb),
                 _ptr(ret), _ptr(adv), ctypes.c_void_p(stream)))
    return ret, adv


def gae_shared(rewards, values, done, gamma, lamb, out_ret=None, out_adv=None):
    """gae() with one value per env shared by its agents (fjsp_gae_shared): rewards f64
    [T, A, N], values f32 [T + 1, N] (row T = the bootstrap value), done u8/bool [T, N] ->
    ret, adv f64 [T, A, N]."""
    T, A, N = rewards.shape
    if values.dtype != torch.float32 or tuple(values.shape) != (T + 1, N) or tuple(done.shape) != (T, N):
        raise ValueError("gae_shared: values f32 [T + 1, N] and done [T, N] expected")
    ret = out_ret if out_ret is not None else torch.empty_like(rewards)
    adv = out_adv if out_adv is not None else torch.empty_like(rewards)
    r = rewards.contiguous(); v = values.contiguous(); d = done.to(torch.uint8).contiguous()
    stream = torch.cuda.current_stream(rewards.device).cuda_stream
    nat.check(nat.lib().fjsp_gae_shared(_ptr(r), _ptr(v), _ptr(d), T, N, A, float(gamma), float(lamb),
                                        _ptr(ret), _ptr(adv), ctypes.c_void_p(stream)))
    return ret, adv


__all__ = ["FJSPVecEnv", "Buffers", "gae", "gae_shared", "AGENTS"]
