"""The reference's TRAINED policy (checkpoints/model.pt, carried as tests/golden/trained_policy.npz
by tests/golden/gen_trained_golden.py) on the GPU path.

* fjsp_a2c_policy (the fused MFMA predict) with the trained weights, greedy, on every state of
  the reference's own test() rollouts (a2c.py:539-645): actions equal the reference's
  predict(deterministic=True), values within 1e-5 relative, masked probabilities equal the
  PyTorch path within 1e-5 (fp32; the fixture's smallest top-2 margin is 5e-5, so no state is
  a near-tie).
* VecMultiAgentA2C.test() with the trained weights on FJSPVecEnv: per env the greedy actions,
  episode length and per-agent reward sums equal the reference's test() (same seeds), and a
  512-env test() replays on the oracle (per-agent reward sums bit-equal)."""
import importlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import parity_util as P  # noqa: E402

SEEDS = [0, 1, 2, 3, 4, 5, 6, 7]


@pytest.fixture(scope="module")
def M():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from tests import gpu_util  # noqa: F401
    A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
    return {"A": A, "V": importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env"),
            "z": np.load(f"{P.GOLDEN}/trained_policy.npz"),
            "ck": A.load_npz_weights(f"{P.GOLDEN}/trained_policy.npz")}


def _learner(M, n):
    L = M["A"].VecMultiAgentA2C(M["V"].FJSPVecEnv(n), batch_size=8, seed=0, use_graph=False)
    L.load_state_dicts(M["ck"])
    return L


def test_fused_policy_trained_matches_reference(M):
    A, z = M["A"], M["z"]
    feats = np.concatenate([z[f"s{s}_gstate"] for s in SEEDS]).T                  # [38, S]
    masks = np.concatenate([z[f"s{s}_masks"] for s in SEEDS]).T
    acts = np.concatenate([z[f"s{s}_actions"] for s in SEEDS]).T                  # [8, S]
    vals = np.concatenate([z[f"s{s}_values"] for s in SEEDS])
    S = feats.shape[1]
    L = _learner(M, 64)
    f = torch.from_numpy(np.ascontiguousarray(feats)).cuda()
    m = torch.from_numpy(np.ascontiguousarray(masks)).cuda()
    act = torch.zeros(8, S, dtype=torch.uint8, device="cuda")
    val = torch.zeros(S, dtype=torch.float32, device="cuda")
    probs = torch.zeros(8, 8, S, dtype=torch.float32, device="cuda")
    L.policy_fused(f, m, 0, True, act, val, probs)
    act_t, pm_t, v_t = L.policy(f, m, deterministic=True)
    torch.cuda.synchronize()
    assert np.array_equal(act.cpu().numpy(), acts)
    assert np.allclose(val.cpu().numpy(), vals, rtol=1e-5, atol=1e-5), float(np.abs(val.cpu().numpy() - vals).max())
    assert np.array_equal(act_t.cpu().numpy(), acts)
    assert torch.allclose(probs, pm_t, atol=1e-5)


@pytest.mark.parametrize("num_orders,seeds", [(5, [0, 1, 2, 3]), (25, [4, 5]), (2, [6, 7])])
def test_trained_test_rollout_matches_reference(M, num_orders, seeds):
    z = M["z"]
    L = _learner(M, 64)
    env = M["V"].FJSPVecEnv(len(seeds))
    res = L.test(num_orders=num_orders, max_steps=500, seeds=seeds, deterministic=True, trace=True, env=env)
    for i, s in enumerate(seeds):
        meta = z[f"s{s}_meta"]
        steps = int(meta[1])
        assert int(res["steps"][i]) == steps, s
        assert np.array_equal(res["actions"][:steps, :, i], z[f"s{s}_actions"]), s
        assert int(res["orders_completed"][i]) == int(meta[2]) and int(res["products_packaged"][i]) == int(meta[3])
        ref_sum = np.cumsum(z[f"s{s}_rewards"], axis=0)[-1]
        assert res["rewards_by_agent"][:, i].tobytes() == ref_sum.tobytes(), s


def test_trained_test_rollout_512_envs_replays_on_oracle(M):
    L = _learner(M, 64)
    n = 512
    env = M["V"].FJSPVecEnv(n)
    seeds = np.arange(n) + 1000
    res = L.test(num_orders=5, max_steps=500, seeds=torch.from_numpy(seeds), deterministic=True, trace=True, env=env)
    acts = res["actions"]
    for e in (0, 131, 511):
        o = O.OracleEnv()
        o.reset(seed=int(seeds[e]), num_orders=5)
        tot = np.zeros(8)
        for t in range(int(res["steps"][e])):
            r = o.step(acts[t, :, e])
            tot += r["rewards"]
        assert res["rewards_by_agent"][:, e].tobytes() == tot.tobytes(), e
        assert bool(r["term"] or r["trunc"]), e
