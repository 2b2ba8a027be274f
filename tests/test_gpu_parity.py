"""GPU parity: the HIP kernels (through the C-ABI) against the reference's golden fixtures and
the CPU oracle.  Bit-exact for every integer field and for the fp64 rewards / GAE."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import parity_util as P  # noqa: E402


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from tests import gpu_util
    return gpu_util


def _groups(traces):
    groups = {}
    for tr in traces:
        key = (tuple(sorted(tr.cfg.items())), tr.num_orders)
        groups.setdefault(key, []).append(tr)
    return groups


def _replay_group(G, trs):
    cfg = dict(trs[0].cfg)
    n = len(trs)
    env = G.make_env(n, **cfg)
    seeds = torch.tensor([tr.seed for tr in trs], dtype=torch.int64)
    b = env.reset(seeds=seeds, num_orders=trs[0].num_orders)
    r = G.to_np(b)
    for i, tr in enumerate(trs):
        assert P.bits_equal(r["obs_i32"][0, i], tr.init_i32), tr.name
        assert P.bits_equal(r["masks"][0, i], tr.init_masks), tr.name
    T = min(tr.steps for tr in trs)
    acts = np.stack([tr.actions[:T] for tr in trs], axis=2)   # [T, 8, n]
    acts_d = torch.from_numpy(np.ascontiguousarray(acts)).cuda()
    for t in range(T):
        b = env.step(acts_d[t], autoreset=True)
        r = G.to_np(b)
        for i, tr in enumerate(trs):
            for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "results"):
                assert P.bits_equal(r[k][0, i], getattr(tr, k)[t]), (tr.name, t, k, r[k][0, i], getattr(tr, k)[t])
            assert r["term"][0, i] == tr.term[t] and r["trunc"][0, i] == tr.trunc[t], (tr.name, t)
            assert r["orders_completed"][0, i] == tr.orders_completed[t], (tr.name, t)
            assert r["packaged"][0, i] == tr.packaged[t], (tr.name, t)
            assert r["sim_time"][0, i] == tr.sim_time[t], (tr.name, t)
            assert P.bits_equal(r["next_i32"][0, i], tr.reset_i32[t]), (tr.name, t, "reset obs")
            assert P.bits_equal(r["next_masks"][0, i], tr.reset_masks[t]), (tr.name, t, "reset masks")
            assert r["status"][0, i] & 1 == 0


def test_golden_traces(G):
    for key, trs in _groups(P.load_traces()).items():
        _replay_group(G, trs)


def test_golden_scenarios(G):
    for key, trs in _groups(P.load_scenarios()).items():
        _replay_group(G, trs)


def test_digests_fused_rollout(G):
    """256 envs x 1000 steps of the fused kernel with on-device actions vs the reference's digests."""
    dg = P.load_digests()
    n, steps, chunk = dg["n_envs"], dg["steps"], dg["chunk"]
    env = G.make_env(n)
    env.reset(seeds=torch.arange(n), num_orders=dg["num_orders"])
    b = env.rollout(steps, action_seed=dg["action_seed"], step0=0, masked=False)
    r = G.to_np(b)
    for e in range(n):
        row = P.chunk_digests(lambda t: (r["obs_i32"][t, e], r["obs_i8"][t, e], r["obs_f32"][t, e],
                                         r["masks"][t, e], r["rewards"][t, e], r["term"][t, e],
                                         r["trunc"][t, e]), steps, chunk)
        assert row == dg["digests"][e], e


@pytest.mark.parametrize("masked", [False, True])
def test_fused_vs_oracle(G, masked):
    """1024 envs x 400 steps, every field bit-exact against the oracle's event-heap restatement."""
    n, steps, seed = 1024, 400, 12345
    env = G.make_env(n)
    env.reset(seeds=torch.arange(n) + 1000, num_orders=30)
    b = env.rollout(steps, action_seed=seed, masked=masked, infos=True)
    r = G.to_np(b)
    rec, _, _ = O.rollout(n, steps, seeds=np.arange(n) + 1000, gid0=0, num_orders=30, action_seed=seed,
                          policy=1 if masked else 0)
    for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "results"):
        assert P.bits_equal(r[k], rec[k]), k
    for k in ("term", "trunc", "orders_completed", "packaged"):
        assert np.array_equal(r[k], rec[k]), k


def test_step_vs_fused(G):
    """k_step with host-supplied actions == k_step_many with on-device actions."""
    n, steps = 512, 120
    a = G.make_env(n)
    bb = G.make_env(n)
    a.reset(seeds=torch.arange(n), num_orders=30)
    bb.reset(seeds=torch.arange(n), num_orders=30)
    tr = G.to_np(bb.rollout(steps, action_seed=7, masked=True))
    acts = np.zeros((steps, 8, n), np.uint8)
    masks = a.reset(seeds=torch.arange(n), num_orders=30).masks[0].t().cpu().numpy()
    for t in range(steps):
        for e in range(n):
            acts[t, :, e] = O.actions(7, e, t, masks[e])
        r = G.to_np(a.step(torch.from_numpy(acts[t]).cuda()))
        assert P.bits_equal(r["obs_i32"][0], tr["obs_i32"][t]), t
        assert P.bits_equal(r["rewards"][0], tr["rewards"][t]), t
        masks = r["next_masks"][0]


@pytest.mark.parametrize("n", [1, 100, 4133])
def test_step_envs_per_workgroup_byte_equal(G, n):
    """k_step (fjsp_step, one launch per step) on 16-, 32- and 64-env workgroups (option
    "step_envs", default 64) writes the same bytes: 160 steps of random actions with auto-resets,
    partial workgroups (4 133 envs)."""
    steps = 160
    gen = torch.Generator(device="cuda").manual_seed(3)
    nact = torch.tensor([3, 8, 3, 3, 3, 3, 3, 3], dtype=torch.uint8, device="cuda")[:, None]
    acts = [torch.randint(0, 8, (8, n), dtype=torch.uint8, device="cuda", generator=gen) % nact for _ in range(steps)]
    runs = {}
    for epw in (64, 32, 16, 0):
        env = G.make_env(n)
        G.native.check(G.native.lib().fjsp_set_option(env.handle, b"step_envs", epw))
        env.reset(seeds=torch.arange(n), num_orders=30)
        outs = []
        for t in range(steps):
            r = env.step(acts[t])
            outs.append(b"".join(getattr(r, k).cpu().numpy().tobytes() for k in
                                 ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "status")))
        runs[epw] = outs
    for epw in (32, 16, 0):
        for t in range(steps):
            assert runs[epw][t] == runs[64][t], (epw, t)
    assert G.native.lib().fjsp_set_option(env.handle, b"step_envs", 8) != 0


def _pinned_buffers(G, n):
    b = G.vec_env.Buffers(1, n, "cpu", infos=True, next_obs=True)
    for k in G.native.OUT_FIELDS:
        t = getattr(b, k, None)
        if t is not None:
            setattr(b, k, t.pin_memory())
    return b


@pytest.mark.parametrize("n,inline,host_out", [(1, False, False), (1, True, False), (100, False, False),
                                               (4096, False, False), (4096, False, True)])
def test_step_server_equals_step(G, n, inline, host_out):
    """The step server (fjsp_server_*: a resident kernel stepped through a host doorbell) ==
    fjsp_step launch by launch: random, absent and out-of-range actions from pinned host memory
    (inline: the one env's 8 action bytes in the doorbell's cache line, fjsp_server_step_actions),
    auto-resets, every output of every step; other calls on the handle in between (read_env,
    snapshot: the server leaves and is relaunched), a pause past the idle relaunch, the final state;
    inline, also past the 16-bit wrap of the inbox's request tags; host_out: the server writes its
    outputs straight into pinned host memory."""
    import time
    rng = np.random.default_rng(n + inline + 2 * host_out)
    envs = [G.make_env(n), G.make_env(n)]
    for env in envs:
        env.reset(seeds=torch.arange(n) + 3, num_orders=30)
    hb = torch.zeros(8, n, dtype=torch.uint8).pin_memory()
    bs = envs[1].server_start(None if inline else hb, autoreset=True,
                              buffers=_pinned_buffers(G, n) if host_out else
                              G.vec_env.Buffers(1, n, envs[1].device, infos=True, next_obs=True))
    assert envs[1].last_kernel() == "k_step_server"
    bl = G.vec_env.Buffers(1, n, envs[0].device, infos=True, next_obs=True)
    nact = np.array([3, 8, 3, 3, 3, 3, 3, 3]).reshape(8, 1)
    for t in range(420):
        acts = (rng.integers(0, 256, (8, n)) * nact >> 8).astype(np.uint8)
        acts[rng.random((8, n)) < 0.05] = 255
        weird = rng.random((8, n)) < 0.02
        acts[weird] = rng.integers(3, 255, size=weird.sum())
        hb.numpy()[:] = acts
        envs[0].step(torch.from_numpy(acts).cuda(), buffers=bl)
        envs[1].server_step(acts[:, 0] if inline else None)   # returns with its outputs written
        torch.cuda.current_stream().synchronize()   # (a device-wide sync would wait for the resident kernel)
        for k in G.native.OUT_FIELDS:
            x, y = getattr(bl, k, None), getattr(bs, k, None)
            if x is not None:
                assert x.cpu().numpy().tobytes() == y.cpu().numpy().tobytes(), (t, k)
        if t == 150:
            v0, v1 = envs[0].read_env(n - 1), envs[1].read_env(n - 1)   # stops the server
            assert bytes(v0) == bytes(v1)
        if t == 300:
            assert torch.equal(envs[0].snapshot(), envs[1].snapshot())
        if t == 350:
            time.sleep(0.02)                                             # past the idle relaunch and exit
    if inline:   # 66 000 more requests: the tags wrap past 0xFFFF; a fixed action stream on both
        ad = torch.zeros(8, 1, dtype=torch.uint8, device=envs[0].device)
        for t in range(66000):
            a = (t * 2654435761) >> 7 & 0xFF
            row = np.array([a % 3, a % 8, (a >> 3) % 3, (a >> 4) % 3, (a >> 5) % 2, 1, 0, (a >> 6) % 2], np.uint8)
            ad.copy_(torch.from_numpy(row).view(8, 1), non_blocking=False)
            envs[0].step(ad, buffers=bl)
            envs[1].server_step(row)
        torch.cuda.current_stream().synchronize()
        for k in G.native.OUT_FIELDS:
            x, y = getattr(bl, k, None), getattr(bs, k, None)
            if x is not None:
                assert x.cpu().numpy().tobytes() == y.cpu().numpy().tobytes(), ("wrap", k)
    envs[1].server_stop()
    assert torch.equal(envs[0].snapshot(), envs[1].snapshot())


def test_agent_order_and_absent_agents(G):
    """Non-canonical dict order and missing agents against the oracle (FJSPSimulation.py:172-205)."""
    n, steps = 64, 200
    rng = np.random.default_rng(3)
    env = G.make_env(n)
    env.reset(seeds=torch.arange(n), num_orders=30)
    oracles = [O.OracleEnv() for _ in range(n)]
    for e, o in enumerate(oracles):
        o.reset(seed=e, num_orders=30)
    for t in range(steps):
        order = rng.permutation(8).astype(np.uint8)
        acts = np.stack([O.actions(99, e, t) for e in range(n)], 1).astype(np.uint8)   # [8, n]
        absent = rng.random((8, n)) < 0.1
        acts[absent] = 255
        weird = rng.random((8, n)) < 0.03
        acts[weird] = rng.integers(3, 255, size=weird.sum())
        r = G.to_np(env.step(torch.from_numpy(acts).cuda(), agent_order=order.tolist()))
        for e in range(n):
            ro = oracles[e].step(acts[:, e], order=order)
            for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "results"):
                assert P.bits_equal(r[k][0, e], ro[k]), (t, e, k, r[k][0, e], ro[k])
            if ro["term"] or ro["trunc"]:
                oracles[e].reset(num_orders=30)


def test_gae_golden(G):
    d = np.load(f"{P.GOLDEN}/gae.npz")
    for c in range(3):
        g, l = d[f"c{c}_gamma_lamb"]
        rw, v, boots, se = d[f"c{c}_rewards"], d[f"c{c}_values"], d[f"c{c}_boots"], d[f"c{c}_seg_end"]
        T = rw.shape[0]
        # segments end at episode ends (next value 0) and at the batch end (bootstrap)
        done = se.copy()
        done[-1] = 0
        ret, adv = G.vec_env.gae(torch.from_numpy(rw).cuda(), torch.from_numpy(v).cuda(),
                                 torch.from_numpy(done.reshape(T, 1)).cuda(),
                                 torch.from_numpy(boots[-1].astype(np.float64)).cuda(), g, l)
        assert P.bits_equal(ret.cpu().numpy(), d[f"c{c}_returns"]), c
        assert P.bits_equal(adv.cpu().numpy(), d[f"c{c}_adv"]), c


def test_gae_vs_oracle_large(G):
    """T=256, 4096 envs x 8 agents with episode boundaries: bit-exact vs the oracle scan."""
    T, N = 256, 4096
    M = 8 * N
    rng = np.random.default_rng(11)
    rw = np.round(rng.normal(0, 3, size=(T, M)) * 8) / 8
    v = rng.normal(0, 5, size=(T, M)).astype(np.float32)
    done = (rng.random((T, N)) < 0.01).astype(np.uint8)
    boot = rng.normal(0, 5, size=M)
    ret, adv = G.vec_env.gae(torch.from_numpy(rw).cuda(), torch.from_numpy(v).cuda(), torch.from_numpy(done).cuda(),
                             torch.from_numpy(boot).cuda(), 0.99, 0.95)
    ret, adv = ret.cpu().numpy(), adv.cpu().numpy()
    cols = rng.choice(M, 64, replace=False)
    for m in cols:
        e = m % N
        se = done[:, e].copy()
        se[-1] = 1
        nseg = int(se.sum())
        boots = np.zeros(nseg)
        if not done[-1, e]:
            boots[-1] = boot[m]
        rr, aa = O.gae(rw[:, m:m + 1], v[:, m:m + 1], boots.reshape(-1, 1), se, 0.99, 0.95)
        assert P.bits_equal(ret[:, m], rr[:, 0]), m
        assert P.bits_equal(adv[:, m], aa[:, 0]), m


@pytest.mark.parametrize("T,N", [(256, 4096), (1, 70), (15, 64), (16, 130), (17, 1), (33, 257), (200, 1000),
                                 (33, 128), (1, 64), (48, 192), (256, 32768)])
def test_gae_shared_equals_gae(G, T, N):
    """fjsp_gae_shared (one value per env shared by its 8 agents, bootstrap = row T; the A2C's
    call) == fjsp_gae over the expanded values, bit for bit, for batch lengths around the
    kernel's 16-step load batches; and the generic scan == the oracle on sampled columns."""
    A = 8
    g = torch.Generator().manual_seed(T * 1000 + N)
    rw = (torch.randn(T, A, N, generator=g, dtype=torch.float64) * 24).round() / 8
    v = torch.randn(T + 1, N, generator=g) * 5
    done = (torch.rand(T, N, generator=g) < 0.02).to(torch.uint8)
    done[T // 2, : N // 3] = 1
    ret_s, adv_s = G.vec_env.gae_shared(rw.cuda(), v.cuda(), done.cuda(), 0.99, 0.95)
    vx = v[:T, None, :].expand(T, A, N).reshape(T, A * N).contiguous()
    boot = v[T].double()[None, :].expand(A, N).reshape(-1).contiguous()
    ret, adv = G.vec_env.gae(rw.reshape(T, A * N).cuda(), vx.cuda(), done.cuda(), boot.cuda(), 0.99, 0.95)
    assert torch.equal(ret_s.reshape(T, A * N).cpu(), ret.cpu())
    assert torch.equal(adv_s.reshape(T, A * N).cpu(), adv.cpu())
    ret, adv = ret.cpu().numpy(), adv.cpu().numpy()
    rwn, vn, dn = rw.reshape(T, A * N).numpy(), vx.numpy(), done.numpy()
    for m in np.random.default_rng(T + N).choice(A * N, min(16, A * N), replace=False):
        e = m % N
        se = dn[:, e].copy()
        se[-1] = 1
        boots = np.zeros(int(se.sum()))
        if not dn[-1, e]:
            boots[-1] = float(boot[m])
        rr, aa = O.gae(rwn[:, m:m + 1], vn[:, m:m + 1], boots.reshape(-1, 1), se, 0.99, 0.95)
        assert P.bits_equal(ret[:, m], rr[:, 0]), m
        assert P.bits_equal(adv[:, m], aa[:, 0]), m


def test_reset_tables_and_read_env(G):
    d = np.load(f"{P.GOLDEN}/reset_tables.npz")
    n = 256
    env = G.make_env(n)
    env.reset(seeds=torch.arange(n), num_orders=30)
    for s in range(0, n, 17):
        v = env.read_env(s)
        o = np.array(v.orders[:30], np.uint32)
        got = np.stack([o & 15, (o >> 4) & 3, (o >> 6) & 3], 1).astype(np.uint8)
        assert np.array_equal(got, d["seeded"][s]), s
        assert v.num_orders == 30 and v.current_step == 0


def test_mt_exchange_matches_numpy(G):
    """fjsp_mt_set/get + reset consume numpy's global stream exactly (FJSPSimulation.py:107-112)."""
    env = G.make_env(3)
    for s in (0, 5, 2**31 + 7):
        rs = np.random.RandomState(s)
        rs.randint(0, 100, size=int(s % 700))   # arbitrary position inside a block
        st = rs.get_state()
        env.mt_set(1, st[1], st[2])
        env.reset(seeds=None, env_mask=torch.tensor([0, 1, 0], dtype=torch.uint8), num_orders=25)
        exp = [(rs.randint(1, 10), rs.randint(0, 3) + 1, rs.randint(0, 3) + 1) for _ in range(25)]
        v = env.read_env(1)
        o = np.array(v.orders[:25], np.uint32)
        got = list(zip((o & 15).tolist(), ((o >> 4) & 3).tolist(), ((o >> 6) & 3).tolist()))
        assert got == exp
        key, pos = env.mt_get(1)
        st2 = rs.get_state()
        assert pos == st2[2] and np.array_equal(key, st2[1])


def test_full_size_properties(G):
    """4096 envs x 1000 steps (the benchmark workload): size-independent invariants plus exact
    parity of a sampled subset of envs against the oracle."""
    n, steps = 4096, 1000
    env = G.make_env(n)
    env.reset(seeds=torch.arange(n), num_orders=30)
    b = env.rollout(steps, action_seed=2024, masked=False)
    torch.cuda.synchronize()
    masks = b.masks
    assert bool((masks[:, [0, 3, 11, 14, 17, 20, 23, 26], :] == 1).all())
    trunc = b.trunc.cpu().numpy()
    # all envs started together and never terminate under random actions -> truncation every 201 steps
    assert np.array_equal(np.nonzero(trunc[:, 0])[0], np.array([200, 401, 602, 803]))
    assert bool((b.trunc[:, 0:1] == b.trunc).all())
    assert int(b.status.bitwise_and(1).sum()) == 0
    # sampled exact parity
    for e in np.arange(0, n, 97)[:8]:
        r1, _, _ = O.rollout(1, steps, seeds=[e], gid0=int(e), num_orders=30, action_seed=2024, policy=0)
        got = b.rewards[:, :, e].cpu().numpy()
        assert P.bits_equal(got, r1["rewards"][:, 0]), e
        got = b.obs_i32[:, :, e].cpu().numpy()
        assert P.bits_equal(got, r1["obs_i32"][:, 0]), e


def test_fused_lds_matches_global_tables(G):
    """The LDS-staged fused kernel and the global-table variant produce identical bytes."""
    n, steps = 2048, 450
    outs = []
    for lds in (0, 1):
        env = G.make_env(n)
        G.native.check(G.native.lib().fjsp_set_option(env.handle, b"fused_lds", lds))
        env.reset(seeds=torch.arange(n) * 7, num_orders=12)
        r1 = G.to_np(env.rollout(steps // 2, action_seed=3, masked=True, infos=True))
        r2 = G.to_np(env.rollout(steps - steps // 2, action_seed=3, step0=steps // 2, masked=True, infos=True))
        outs.append((r1, r2))
    for k in outs[0][0]:
        assert P.bits_equal(outs[0][0][k], outs[1][0][k]), k
        assert P.bits_equal(outs[0][1][k], outs[1][1][k]), k


def test_staged_stores_match_direct_stores(G):
    """The LDS-staged wide-store path (lean outputs) writes the same bytes as direct stores and
    as the full-output kernel."""
    n, steps = 1024, 300
    outs = []
    for staged, infos in ((1, False), (0, False), (1, True)):   # staged is opt-in (default off)
        env = G.make_env(n)
        G.native.check(G.native.lib().fjsp_set_option(env.handle, b"staged_stores", staged))
        env.reset(seeds=torch.arange(n) + 5, num_orders=20)
        outs.append(G.to_np(env.rollout(steps, action_seed=11, masked=bool(staged), infos=infos)))
    # staged (masked) vs full (masked) must agree exactly; unmasked run checked against the oracle
    for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "status"):
        assert P.bits_equal(outs[0][k], outs[2][k]), k
    rec, _, _ = O.rollout(n, steps, seeds=np.arange(n) + 5, gid0=0, num_orders=20, action_seed=11, policy=0)
    for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards"):
        assert P.bits_equal(outs[1][k], rec[k]), k


@pytest.mark.parametrize("policy", ["random", "masked", "heuristic"])
def test_pipelined_matches_single_wave(G, policy):
    """The two-wave pipelined k_step_pipe (default for lean outputs) writes the same bytes and
    leaves the same state as the single-wave k_step_many; N not a multiple of 64."""
    n, steps = 1000, 333
    outs = []
    for pipe, lds in ((1, -1), (0, 0), (1, 0)):
        env = G.make_env(n)
        G.native.check(G.native.lib().fjsp_set_option(env.handle, b"pipeline", pipe))
        G.native.check(G.native.lib().fjsp_set_option(env.handle, b"fused_lds", lds))
        env.reset(seeds=torch.arange(n) * 3 + 1, num_orders=5 if policy == "heuristic" else 20)
        r1 = G.to_np(env.rollout(steps, action_seed=21, policy=policy))
        r2 = G.to_np(env.rollout(7, action_seed=21, step0=steps, policy=policy, infos=True))   # full path after
        outs.append((r1, r2))
    for o in outs[1:]:
        for k in outs[0][0]:
            assert P.bits_equal(outs[0][0][k], o[0][k]), k
        for k in outs[0][1]:
            assert P.bits_equal(outs[0][1][k], o[1][k]), k


def test_pipelined_single_emit_wave_large_n(G):
    """N > 16384 takes the one-emit-wave pipelined variant (global tables): same bytes as the
    single-wave kernel."""
    n, steps = 16448, 60
    outs = []
    for pipe in (1, 0):
        env = G.make_env(n)
        G.native.check(G.native.lib().fjsp_set_option(env.handle, b"pipeline", pipe))
        env.reset(seeds=torch.arange(n), num_orders=10)
        outs.append(G.to_np(env.rollout(steps, action_seed=8, masked=True)))
        if pipe:
            assert env.last_kernel() == "k_step_pipe<1emit>"
    for k in outs[0]:
        assert P.bits_equal(outs[0][k], outs[1][k]), k
