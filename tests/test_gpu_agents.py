"""Agent-group pipeline (k_step_ag, the default kernel for uniform-random actions with LDS
tables and auto-reset): the AGV and the machines, the packaging stations and the pickup station
run on different wavefronts of the env's workgroup.  Its outputs and end state must be the
bytes of the other kernels and of the oracle (FJSPSimulation.step / reset(seed=None) with the
SimPy event heap), across launch boundaries, truncations, all-orders-done resets, configurations
and partial workgroups."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import parity_util as P  # noqa: E402

LEAN = ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "status")
AG = "k_step_ag<lds,predraw>"               # outputs from the core workgroup's emit waves (default)


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from tests import gpu_util
    return gpu_util


def _env(G, n, agents, pipeline=1, **cfg):
    env = G.make_env(n, **cfg)
    lib = G.native.lib()
    G.native.check(lib.fjsp_set_option(env.handle, b"agents", agents))
    G.native.check(lib.fjsp_set_option(env.handle, b"pipeline", pipeline))
    return env


def _chunks(G, env, chunks, seed, t0=0):
    """Lean uniform-random rollouts in launches of the given sizes, concatenated along time."""
    parts, t = [], t0
    for k in chunks:
        parts.append(G.to_np(env.rollout(k, action_seed=seed, step0=t, policy="random")))
        t += k
    return {key: np.concatenate([p[key] for p in parts]) for key in parts[0]}


def _views(env, es):
    """fjsp_read_env fields + the live MT19937 stream of the given envs."""
    out = []
    for e in es:
        v = env.read_env(e)
        fields = tuple(tuple(getattr(v, f)) if f == "orders" else getattr(v, f) for f, _ in v._fields_)
        out.append((fields, env.mt_get(e)))
    return out


def _same_views(a, b):
    for (va, (ka, pa)), (vb, (kb, pb)) in zip(a, b):
        assert va == vb
        assert pa == pb and np.array_equal(ka, kb)


def test_agents_matches_other_kernels_and_oracle(G):
    """1000 envs (a partial workgroup), 20 orders, launches of 1..200 steps: k_step_ag == k_step_pipe == k_step_many == the
    oracle, and the state left behind is the same (a full-output step after it, the env views,
    the MT streams)."""
    n, seeds, chunks = 1000, np.arange(1000) * 3 + 1, [1, 37, 200, 5, 120, 2]
    runs = []
    for agents, pipeline in ((1, 1), (0, 1), (0, 0)):
        env = _env(G, n, agents, pipeline)
        env.reset(seeds=torch.from_numpy(seeds), num_orders=20)
        a = _chunks(G, env, chunks, seed=21)
        if agents:
            assert env.last_kernel() == AG
        tail = G.to_np(env.rollout(3, action_seed=21, step0=sum(chunks), policy="random", infos=True))
        runs.append((a, tail, _views(env, (0, 63, 64, 500, 999))))
    for a, tail, views in runs[1:]:
        for k in LEAN:
            assert P.bits_equal(runs[0][0][k], a[k]), k
        for k in runs[0][1]:
            assert P.bits_equal(runs[0][1][k], tail[k]), k
        _same_views(runs[0][2], views)
    rec, _, _ = O.rollout(n, sum(chunks), seeds=seeds, num_orders=20, action_seed=21, policy=0)
    a = runs[0][0]
    for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards"):
        assert P.bits_equal(a[k], rec[k]), k
    assert np.array_equal(a["term"], rec["term"]) and np.array_equal(a["trunc"], rec["trunc"])


def test_agents_two_rounds_of_workgroups(G):
    """Above 16 384 envs (here 20 000: 313 workgroups of 64 envs, two rounds on 256 CUs, the last
    one partial) k_step_ag runs as well: bytes equal to k_step_pipe<1emit> over launches with
    truncation resets every 51 steps, and the env views / MT streams left behind are equal."""
    n, chunks = 20000, [120, 1, 77]
    runs = []
    for agents in (1, 0):
        env = _env(G, n, agents, 1, max_episode_steps=50)
        env.reset(seeds=torch.arange(n) * 5 + 3, num_orders=10)
        a = _chunks(G, env, chunks, seed=33)
        assert env.last_kernel() == (AG if agents else "k_step_pipe<1emit>")
        runs.append((a, _views(env, (0, 16383, 16384, 19999))))
    for k in LEAN:
        assert P.bits_equal(runs[0][0][k], runs[1][0][k]), k
    assert (runs[0][0]["trunc"].sum() > n)
    _same_views(runs[0][1], runs[1][1])
    # sampled envs of the first round, of the second round and of its partial last workgroup
    # against the oracle at their ids (k_step_ag's own direct pin in this regime)
    got = runs[0][0]
    for e0 in (0, 16380, 19992):
        rec, _, _ = O.rollout(8, sum(chunks), seeds=np.arange(e0, e0 + 8) * 5 + 3, gid0=e0, num_orders=10,
                              action_seed=33, policy=0, max_episode_steps=50)
        for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards"):
            assert P.bits_equal(got[k][:, e0:e0 + 8], rec[k]), (e0, k)
        assert np.array_equal(got["trunc"][:, e0:e0 + 8], rec["trunc"]), e0


def test_agents_all_orders_done_resets(G):
    """One order per episode: random play completes it in ~1 of 4 episodes, so episodes end by
    termination (K's completion count -> AM's reset at the next step) and by truncation, at
    scattered steps; bytes equal to k_step_pipe and the oracle."""
    n, steps = 2048, 700
    seeds = np.arange(n) + 100
    runs = []
    for agents in (1, 0):
        env = _env(G, n, agents)
        env.reset(seeds=torch.from_numpy(seeds), num_orders=1)
        runs.append(_chunks(G, env, [300, 1, 399], seed=5))
    for r in runs[1:]:
        for k in LEAN:
            assert P.bits_equal(runs[0][k], r[k]), k
    assert runs[0]["term"].sum() > 100, "the test needs all-orders-done resets"
    rec, _, _ = O.rollout(n, steps, seeds=seeds, num_orders=1, action_seed=5, policy=0)
    for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards"):
        assert P.bits_equal(runs[0][k], rec[k]), k
    assert np.array_equal(runs[0]["term"], rec["term"])


@pytest.mark.parametrize("cfg,num_orders", [
    (dict(max_episode_steps=25), 4),                       # a truncation every 26 steps
    (dict(pt_packaging=10), 2),                            # packaging completes the next step
    (dict(tray_capacity=2, mask_tray_capacity=2), 6),      # many trays, slot arena pressure
    (dict(storage_capacity=2, packaging_capacity=3), 8),   # storage full, packaging Resource waits
    (dict(pt_small=10, pt_big=20), 3),                     # short machine runs: grants every step
    ({}, 0),                                               # empty order tables
    ({}, 64),                                              # the largest order table
])
def test_agents_configs(G, cfg, num_orders):
    """Non-default configurations: k_step_ag == k_step_pipe (statuses included) == the oracle."""
    n, chunks = 320, [60, 1, 139]
    seeds = np.arange(n) * 11 + 2
    runs = []
    for agents in (1, 0):
        env = _env(G, n, agents, **cfg)
        env.reset(seeds=torch.from_numpy(seeds), num_orders=num_orders)
        runs.append((_chunks(G, env, chunks, seed=13), _views(env, (0, 100, 319))))
    for k in LEAN:
        assert P.bits_equal(runs[0][0][k], runs[1][0][k]), (cfg, k)
    _same_views(runs[0][1], runs[1][1])
    rec, _, _ = O.rollout(n, sum(chunks), seeds=seeds, num_orders=num_orders, action_seed=13, policy=0, **cfg)
    diverged = (runs[0][0]["status"] & 1).astype(bool)   # paths the closed form flags (not emulated)
    # the flagged env-steps are exactly the ones the oracle's event heap marks as leaving the
    # reference's normal path (a packaging Request that waits, the reference raising, an int8
    # observation overflow), and only the Resource-wait configuration has any
    o_div = (np.asarray(rec["status"]) & (O.ST_EXCEPTION | O.ST_PKG_WAIT | O.ST_OBS_OVERFLOW)) != 0
    assert np.array_equal(diverged, o_div), cfg
    n_steps, n_envs = int(diverged.sum()), int(diverged.any(0).sum())
    print(f"test_agents_configs {cfg} num_orders={num_orders}: DIVERGED {n_steps} of {diverged.size} env-steps, "
          f"{n_envs} of {n} envs excluded from the oracle comparison")
    if cfg.get("packaging_capacity", 20) >= 20:
        assert n_steps == 0, cfg
    for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards"):
        got, want = runs[0][0][k], rec[k]
        ok = ~diverged
        assert P.bits_equal(got[ok], want[ok]), (cfg, k)


def test_agents_staggered_masked_resets(G):
    """Explicit masked resets between launches (episodes of every age in one workgroup) and short
    episodes: k_step_ag == k_step_pipe."""
    n = 384
    outs = []
    for agents in (1, 0):
        env = _env(G, n, agents, max_episode_steps=37)
        env.reset(seeds=torch.arange(n) + 11, num_orders=3)
        seq = []
        for i, k in enumerate((13, 29, 8, 50)):
            seq.append(G.to_np(env.rollout(k, action_seed=4, step0=100 * i, policy="random")))
            mask = ((torch.arange(n) % (i + 2)) == 0).to(torch.uint8).to(env.device)
            env.reset(env_mask=mask, num_orders=3)
        seq.append(_chunks(G, env, [90, 45, 120], seed=6))
        outs.append(seq)
    for i, (x, y) in enumerate(zip(*outs)):
        for k in x:
            assert P.bits_equal(x[k], y[k]), (i, k)


def test_agents_full_size_invariants(G):
    """The bench workload (4096 envs, 30 orders, 1000 steps in 200-step launches):
    k_step_ag == k_step_pipe, plus sampled envs exact against the
    oracle."""
    n = 4096
    runs = []
    for agents in (1, 0):
        env = _env(G, n, agents)
        env.reset(seeds=torch.arange(n), num_orders=30)
        runs.append(_chunks(G, env, [200] * 5, seed=0))
        if agents:
            assert env.last_kernel() == AG
    for r in runs[1:]:
        for k in LEAN:
            assert P.bits_equal(runs[0][k], r[k]), k
    sample = np.array([0, 1, 2047, 4095])
    for gid in sample:
        rec, _, _ = O.rollout(1, 1000, seeds=np.array([gid]), gid0=int(gid), num_orders=30, action_seed=0, policy=0)
        for k in ("obs_i32", "masks", "rewards"):
            assert P.bits_equal(runs[0][k][:, gid:gid + 1], rec[k]), (gid, k)


@pytest.mark.parametrize("n", [250, 1001])
def test_agents_byte_rows_not_quad_aligned(G, n):
    """Env counts that are not a multiple of 4 or of the 64-env workgroup (byte rows at odd
    offsets, a partial last workgroup): k_step_ag == k_step_pipe."""
    runs = []
    for agents in (1, 0):
        env = _env(G, n, agents)
        env.reset(seeds=torch.arange(n) + 9, num_orders=4)
        runs.append(_chunks(G, env, [70, 1, 60], seed=8))
        if agents:
            assert env.last_kernel() == AG
    for k in LEAN:
        assert P.bits_equal(runs[0][k], runs[1][k]), k


@pytest.mark.parametrize("epw", [16, 32, 64])
def test_agents_envs_per_workgroup(G, epw):
    """k_step_ag with 16 / 32 / 64 envs per workgroup ("ag_envs"; 1000 envs leave a partial last
    workgroup in each layout): the bytes of k_step_pipe, launch boundaries and end state included."""
    n, seeds, chunks = 1000, np.arange(1000) * 5 + 2, [1, 37, 200, 5, 120]
    runs = []
    for agents in (1, 0):
        env = _env(G, n, agents)
        G.native.check(G.native.lib().fjsp_set_option(env.handle, b"ag_envs", epw))
        env.reset(seeds=torch.from_numpy(seeds), num_orders=30)
        a = _chunks(G, env, chunks, seed=9)
        if agents:
            assert env.last_kernel() == AG
        runs.append((a, _views(env, (0, 15, 16, 31, 32, 63, 64, 999))))
    for k in LEAN:
        assert P.bits_equal(runs[0][0][k], runs[1][0][k]), k
    _same_views(runs[0][1], runs[1][1])


@pytest.mark.parametrize("agents", [1, 0])
def test_bounded_handoff_waits(G, agents):
    """The hand-off waits of the multi-wave kernels (k_step_ag's flag spins, k_step_pipe's
    mailboxes) are bounded.  At the default bound a 4 096-env x 1 024-step bench launch never
    gives up (fault word 0, no env carries FJSP_STATUS_SPIN_TIMEOUT).  At the smallest bound (256
    sleeps, ~7 us: the first step waits that long for the tables' copy-in) a wait may give up:
    the launch still ends, and a workgroup that gave up
    flags every env it holds (status bit 0x80 | DIVERGED, fault word bit 0) while workgroups that
    did not are byte-identical to the unbounded run; with one workgroup's owner wave held back
    (option "test_stall") the give-up path provably runs."""
    env = _env(G, 4096, agents)
    env.reset(num_orders=30)
    st = G.to_np(env.rollout(1024, action_seed=3, policy="random"))["status"]
    torch.cuda.synchronize()
    assert env.last_kernel() == (AG if agents else "k_step_pipe<lds,2emit,predraw>")
    assert env.faults() == 0 and not (st & 0x80).any()
    n = 256
    ref = _env(G, n, agents)
    ref.reset(num_orders=30)
    r0 = G.to_np(ref.rollout(64, action_seed=5, policy="random"))
    tight = _env(G, n, agents)
    G.native.check(G.native.lib().fjsp_set_option(tight.handle, b"spin_cap", 256))
    tight.reset(num_orders=30)
    r1 = G.to_np(tight.rollout(64, action_seed=5, policy="random"))
    fault = tight.faults(clear=True)
    flagged = (r1["status"][-1] & 0x80) != 0                      # [n]: the env's workgroup gave up
    assert bool(fault & 1) == bool(flagged.any())
    assert tight.faults() == 0                                    # cleared
    ok = ~flagged
    for k in LEAN:
        if k == "status":
            continue
        assert np.array_equal(r1[k][:, ok], r0[k][:, ok]), k
    if flagged.any():
        assert ((r1["status"][-1][flagged] & 0x81) == 0x81).all()
    # the give-up path itself: workgroup 0's owner wave (k_step_ag's AM, k_step_pipe's sim wave)
    # sleeps ~0.25 ms before its first step (option "test_stall"), far past the 256-sleep bound
    # of the other waves' waits for its first post: they give up, the launch still ends, the fault
    # word says so, and exactly workgroup 0's envs are flagged (env 0 among them); every other
    # env is byte-identical to the unbounded run
    stalled = _env(G, n, agents)
    G.native.check(G.native.lib().fjsp_set_option(stalled.handle, b"spin_cap", 256))
    G.native.check(G.native.lib().fjsp_set_option(stalled.handle, b"test_stall", 64))
    stalled.reset(num_orders=30)
    r2 = G.to_np(stalled.rollout(64, action_seed=5, policy="random"))
    assert stalled.faults() & 1
    flagged = (r2["status"][-1] & 0x80) != 0
    assert flagged[0] and not flagged[64:].any()
    assert ((r2["status"][-1][flagged] & 0x81) == 0x81).all()
    ok = ~flagged
    for k in LEAN:
        if k == "status":
            continue
        assert np.array_equal(r2[k][:, ok], r0[k][:, ok]), k
