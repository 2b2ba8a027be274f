"""Edge cases and invariants of the HIP path (scenario, property and invariant
tests): empty / maximum order tables, a single env, an exhausted tray pool, extreme configs,
API guards, and conservation invariants over long rollouts read back through fjsp_read_env."""
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


@pytest.mark.parametrize("n,num_orders,cfg,masked", [
    (64, 0, {}, True),                                   # empty order table: never terminates
    (64, 64, {}, False),                                 # maximum order table
    (1, 30, {}, True),                                   # a single env
    (96, 20, {"num_trays": 3}, True),                    # tray pool exhausted
    (64, 8, {"tray_capacity": 1, "mask_tray_capacity": 1}, True),
    (64, 5, {"max_episode_steps": 0}, True),             # truncation after every step
    (64, 12, {"storage_capacity": 0}, True),             # every storage drop is lost
    (64, 6, {"step_size": 20, "pt_small": 60, "pt_big": 100, "pt_packaging": 40}, True),
])
def test_edge_configs_vs_oracle(G, n, num_orders, cfg, masked):
    steps = 300
    env = G.make_env(n, **cfg)
    env.reset(seeds=torch.arange(n) + 900, num_orders=num_orders)
    r = G.to_np(env.rollout(steps, action_seed=77, masked=masked, infos=True))
    rec, _, _ = O.rollout(n, steps, seeds=np.arange(n) + 900, num_orders=num_orders, action_seed=77,
                          policy=int(masked), **cfg)
    ok = (rec["status"] & (O.ST_EXCEPTION | O.ST_PKG_WAIT | O.ST_OBS_OVERFLOW)) == 0
    assert ok.all()
    for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "results"):
        assert P.bits_equal(r[k], rec[k]), k
    for k in ("term", "trunc", "orders_completed", "packaged"):
        assert np.array_equal(r[k], rec[k]), k
    if num_orders == 0:
        assert r["term"].sum() == 0


def test_api_guards(G):
    nat = G.native
    env = G.make_env(64)
    with pytest.raises(nat.FjspNativeError):
        env.reset(num_orders=65)
    with pytest.raises(ValueError):
        env.step(torch.zeros(8, 63, dtype=torch.uint8, device=env.device))
    with pytest.raises(nat.FjspNativeError):
        env2 = G.make_env(8)
        env2.rollout(10)                                   # step before reset
    big = G.make_env(1 << 16)
    big.reset(num_orders=1)
    b = G.vec_env.Buffers(1, 1 << 16, big.device, infos=False)
    with pytest.raises(nat.FjspNativeError):               # K * N * 64 B >= 4 GiB (32-bit offsets)
        nat.check(nat.lib().fjsp_step_many(big.handle, 1 << 10, 0, 0, 0, 0, 1, __import__("ctypes").byref(b.struct())))


def test_conservation_invariants(G):
    """Over 1 200 masked-random steps with auto-reset: per order packaged <= processed <= n,
    complete <=> all packaged, orders_completed == #complete, total packaged == sum of packaged
    products, counts never decrease within an episode."""
    n, steps = 512, 1200
    env = G.make_env(n)
    env.reset(seeds=torch.arange(n), num_orders=6)
    sample = list(range(0, n, 37))
    prev = {}
    for chunk in range(12):
        env.rollout(steps // 12, action_seed=3, step0=chunk * (steps // 12), masked=True)
        torch.cuda.synchronize()
        for e in sample:
            v = env.read_env(e)
            orders = [v.orders[i] for i in range(v.num_orders)]
            nprod = [w & 15 for w in orders]
            proc = [(w >> 8) & 15 for w in orders]
            pack = [(w >> 12) & 15 for w in orders]
            comp = [(w >> 16) & 1 for w in orders]
            assert all(pk <= pc <= nn for pk, pc, nn in zip(pack, proc, nprod)), e
            assert all(c == (pk == nn) for c, pk, nn in zip(comp, pack, nprod)), e
            assert v.orders_completed == sum(comp), e
            assert v.total_packaged == sum(pack), e
            assert v.status & 1 == 0, e
            if e in prev and v.current_step > prev[e][0]:   # same episode: monotone counters
                assert v.total_packaged >= prev[e][1] and v.orders_completed >= prev[e][2], e
            prev[e] = (v.current_step, v.total_packaged, v.orders_completed)
