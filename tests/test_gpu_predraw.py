"""Pre-drawn reset tables (k_step_pipe<lds,2emit,predraw>): the pre-draw wave draws each env's
next order table during the episode; an auto-reset then consumes it instead of drawing on the
sim wave.  The results must be the bytes of the inline-reset kernels and of the oracle
(FJSPSimulation.reset(seed=None) continuing the env's MT19937 stream), whatever the episode
lengths, launch boundaries, table sizes or interleaved reset paths."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import parity_util as P  # noqa: E402

LEAN = ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "status")


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from tests import gpu_util
    return gpu_util


def _env(G, n, predraw, **cfg):
    env = G.make_env(n, **cfg)
    G.native.check(G.native.lib().fjsp_set_option(env.handle, b"predraw", predraw))
    return env


def _chunks(G, env, chunks, policy, seed=3):
    """Lean rollouts in launches of the given sizes, concatenated along time."""
    parts, t = [], 0
    for k in chunks:
        parts.append(G.to_np(env.rollout(k, action_seed=seed, step0=t, policy=policy)))
        t += k
    return {key: np.concatenate([p[key] for p in parts]) for key in parts[0]}


@pytest.mark.parametrize("num_orders", [1, 2, 5, 30, 64])
def test_predraw_matches_inline_and_oracle(G, num_orders):
    """Heuristic episodes end at scattered steps (many resets per launch, some right after a
    launch boundary); predraw on == predraw off == the oracle, and the MT streams end equal."""
    n = 200   # not a multiple of 64: a partial workgroup
    chunks = [17, 40, 3, 100, 1, 60, 179]
    seeds = np.arange(n) * 5 + 2
    runs = []
    for predraw in (1, 0):
        env = _env(G, n, predraw)
        env.reset(seeds=torch.from_numpy(seeds), num_orders=num_orders)
        runs.append((_chunks(G, env, chunks, "heuristic"), env))
        if predraw:
            assert env.last_kernel() == "k_step_pipe<lds,2emit,predraw>"
    (a, ea), (b, eb) = runs
    for k in LEAN:
        assert P.bits_equal(a[k], b[k]), k
    steps = sum(chunks)
    rec, _, _ = O.rollout(n, steps, seeds=seeds, num_orders=num_orders, policy=3)
    for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards"):
        assert P.bits_equal(a[k], rec[k]), k
    assert np.array_equal(a["term"], rec["term"]) and np.array_equal(a["trunc"], rec["trunc"])
    assert (a["term"] | a["trunc"]).sum() >= n, "the test needs resets"
    for e in (0, 63, 64, 199):
        ka, pa = ea.mt_get(e)
        kb, pb = eb.mt_get(e)
        assert pa == pb and np.array_equal(ka, kb), e


def test_predraw_synchronised_truncations(G):
    """Random actions: every env truncates at step 201 of each episode (one reset per env per
    201 steps, all lanes together), across launch boundaries; 0 orders (nothing to draw)."""
    n = 256
    for num_orders in (30, 0):
        runs = []
        for predraw in (1, 0):
            env = _env(G, n, predraw)
            env.reset(seeds=torch.arange(n) + 40, num_orders=num_orders)
            runs.append(_chunks(G, env, [150, 150, 200, 150], "random", seed=9))
        for k in LEAN:
            assert P.bits_equal(runs[0][k], runs[1][k]), (num_orders, k)
    rec, _, _ = O.rollout(n, 650, seeds=np.arange(n) + 40, num_orders=0, action_seed=9, policy=0)
    for k in ("obs_i32", "masks", "rewards"):
        assert P.bits_equal(runs[0][k], rec[k]), k


def test_predraw_interleaved_reset_paths(G):
    """Pre-draw launches interleaved with the other reset paths (one-launch-per-step k_step
    auto-reset, full-output k_step_many, explicit continued reset, mt_set): each of them
    invalidates or honours a pending table so that the streams never fork."""
    n = 192
    outs = []
    for predraw in (1, 0):
        env = _env(G, n, predraw)
        env.reset(seeds=torch.arange(n) + 7, num_orders=3)
        seq = [_chunks(G, env, [90], "heuristic")]
        acts = G.vec_env.Buffers(1, n, env.device, infos=True, next_obs=True)
        for t in range(25):   # host-supplied (heuristic-equivalent) actions through k_step
            b = env.rollout(1, action_seed=0, step0=0, policy="heuristic", infos=True)   # full outputs, k_step_many
            seq.append(G.to_np(b))
        seq.append(_chunks(G, env, [70, 5], "heuristic"))
        env.reset(num_orders=3)   # continued stream through k_reset
        seq.append(_chunks(G, env, [120], "heuristic"))
        key, pos = env.mt_get(5)
        env.mt_set(5, key, pos)   # drops env 5's pending table; the stream is unchanged
        seq.append(_chunks(G, env, [140], "heuristic"))
        env.step(torch.zeros(8, n, dtype=torch.uint8, device=env.device), buffers=acts)   # k_step, autoreset
        seq.append(_chunks(G, env, [60], "heuristic"))
        outs.append(seq)
        del acts
    for i, (x, y) in enumerate(zip(*outs)):
        for k in x:
            assert P.bits_equal(x[k], y[k]), (i, k)


def test_predraw_snapshot_restore(G):
    """A snapshot carries the pre-draw state (both MT rows, pending tables): a restored handle
    continues bit-identically, also when the table was finished in an earlier launch."""
    n = 128
    env = _env(G, n, 1)
    env.reset(seeds=torch.arange(n), num_orders=2)
    _chunks(G, env, [130], "heuristic")
    snap = env.snapshot()
    a = _chunks(G, env, [50, 70], "heuristic")
    env2 = _env(G, n, 1)
    env2.restore(snap)
    b = _chunks(G, env2, [50, 70], "heuristic")
    env3 = _env(G, n, 0)
    env3.restore(snap)
    c = _chunks(G, env3, [120], "heuristic")
    for k in LEAN:
        assert P.bits_equal(a[k], b[k]) and P.bits_equal(a[k], c[k]), k


def test_pickup_ahead_desynchronised_episodes(G):
    """Uniform-random actions (emit wave 1 runs each step's pickup ahead of the sim wave):
    lanes whose episodes end at different steps (staggered masked resets, short episodes)
    must match the single-wave kernel, across launch boundaries and resets."""
    n = 320
    cfg = dict(max_episode_steps=37)
    outs = []
    for pipe, predraw in ((1, 1), (0, 0)):
        env = _env(G, n, predraw, **cfg)
        G.native.check(G.native.lib().fjsp_set_option(env.handle, b"pipeline", pipe))
        G.native.check(G.native.lib().fjsp_set_option(env.handle, b"agents", 0))   # k_step_ag: test_gpu_agents.py
        env.reset(seeds=torch.arange(n) + 11, num_orders=3)
        seq = []
        for i, k in enumerate((13, 29, 8, 50)):
            seq.append(G.to_np(env.rollout(k, action_seed=4, step0=100 * i, policy="random")))
            mask = ((torch.arange(n) % (i + 2)) == 0).to(torch.uint8).to(env.device)
            env.reset(env_mask=mask, num_orders=3)   # staggered episode starts
        seq.append(_chunks(G, env, [90, 45, 120], "random", seed=6))
        if pipe:
            assert env.last_kernel() == "k_step_pipe<lds,2emit,predraw>"
        outs.append(seq)
    for i, (x, y) in enumerate(zip(*outs)):
        for k in x:
            assert P.bits_equal(x[k], y[k]), (i, k)
    assert (outs[0][-1]["trunc"].sum(axis=1) > 0).sum() > 5   # truncations spread over many steps
