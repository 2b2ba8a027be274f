"""The batched A2C learner (a2c_vec.py) against the REFERENCE's MultiAgentA2C (fixtures from
tests/golden/gen_a2c_golden.py): initialisation, predict (masked probabilities, greedy actions,
log-probs, values) and one full _update (losses and the parameter step).

Runs on CPU: the learner is plain torch math on whatever device its tensors live on; the
observations of the reference run are rebuilt with the oracle (test infrastructure) from the
recorded actions.  The GPU end-to-end version is tests/test_gpu_a2c.py.

Tolerances (fp32 network math, reference per-sample GEMV vs batched GEMM): values / log-probs
1e-5 absolute, losses 1e-4 relative; Adam's first step is ~lr * sign(grad), so parameters are
compared as delta / lr with 1e-2 absolute, allowing a 1e-3 fraction of elements whose gradient
is within rounding of zero to differ."""
import importlib

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import parity_util as P

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
spec = importlib.import_module("multi-agent-rl-for-fjsp_amd.spec")

HP = dict(gamma=0.99, lamb=0.95, lr_actor=3e-4, lr_critic=1e-3, entropy_coef=0.01, max_grad_norm=0.5)


@pytest.fixture(scope="module")
def gold():
    return np.load(f"{P.GOLDEN}/a2c_golden.npz")


def _params(actors, critic):
    out = {}
    for i, a in enumerate(spec.AGENTS):
        for k, v in actors.actor_state_dict(i).items():
            out[f"actor.{a}.{k}"] = v
    for k, v in critic.state_dict().items():
        out[f"critic.{k}"] = v.detach().cpu()
    return out


def test_init_matches_reference(gold):
    actors, critic = A.init_networks(seed=0)
    for k, v in _params(actors, critic).items():
        assert float(v.double().sum()) == pytest.approx(float(gold[f"init_sum_{k}"]), rel=1e-12, abs=1e-12), k
        assert np.array_equal(v.reshape(-1)[:8].numpy(), gold[f"init_head_{k}"]), k


def test_actor_stack_equals_per_agent_networks():
    torch.manual_seed(3)
    nets = [A.ActorNet(A.OBS_DIMS[a], A.N_ACTIONS[a]) for a in range(8)]
    st = A.ActorStack()
    st.load_actor_nets(nets)
    feats = torch.randn(38, 50) * 3
    probs = st(A.actor_inputs(feats, A.gather_index("cpu")))
    for a in range(8):
        x = feats[A.OBS_OFFS[a]:A.OBS_OFFS[a] + A.OBS_DIMS[a]].t()
        ref = nets[a](x).t()
        n = A.N_ACTIONS[a]
        assert torch.allclose(probs[a, :n], ref, atol=1e-6), a
        assert float(probs[a, n:].abs().max() if n < 8 else 0.0) == 0.0


def _replay_obs(actions, seed=0, num_orders=25):
    """Pre-step observations (features, masks), rewards and done flags of the reference run."""
    idx = spec.a2c_feature_index()
    env = O.OracleEnv()
    r = env.reset(seed=seed, num_orders=num_orders)
    T = len(actions)
    feats = np.zeros((T + 1, 38, 1), np.float32)
    masks = np.zeros((T + 1, 29, 1), np.int8)
    rew = np.zeros((T, 8, 1))
    done = np.zeros((T, 1), np.uint8)

    def put(t, rec):
        flat = np.concatenate([rec["obs_i32"], rec["obs_i8"], rec["obs_f32"]]).astype(np.float32)
        feats[t, :, 0] = flat[idx]
        masks[t, :, 0] = rec["masks"]
    put(0, r)
    for t in range(T):
        r = env.step(actions[t])
        rew[t, :, 0] = r["rewards"]
        done[t, 0] = r["term"] | r["trunc"]
        if done[t, 0]:
            r = env.reset(num_orders=num_orders)
        put(t + 1, r)
    return feats, masks, rew, done


@pytest.mark.parametrize("dedup", [False, True])
@pytest.mark.parametrize("case", ["greedy", "replay"])
def test_predict_and_update_match_reference(gold, case, dedup):
    acts = gold[f"{case}_actions"]
    T = len(acts)
    feats, masks, rew, done = _replay_obs(acts)
    actors, critic = A.init_networks(seed=0)
    before = {k: v.clone() for k, v in _params(actors, critic).items()}
    gidx, midx = A.gather_index("cpu"), A.mask_index("cpu")
    # predict at every step: values, log-probs of the taken actions, greedy actions
    f = torch.from_numpy(feats[:T, :, 0].T.copy())             # [38, T] (steps as the batch)
    m = torch.from_numpy(masks[:T, :, 0].T.copy())
    with torch.no_grad():
        pm = A.masked_probs(actors(A.actor_inputs(f, gidx)), A.agent_masks(m, midx))
        v = critic(f.t()).view(-1)
        lp = A.categorical_log_prob(pm, torch.from_numpy(acts.T.astype(np.int64)))
    assert np.allclose(v.numpy(), gold[f"{case}_values"], atol=1e-5, rtol=1e-5)
    assert np.allclose(lp.numpy().T, gold[f"{case}_logprobs"], atol=1e-5)
    if case == "greedy":
        assert np.array_equal(torch.argmax(pm, dim=1).numpy().T, acts)
    # GAE exactly as the reference (f64 scan over the reference's f32 values; the episode end
    # bootstraps 0, the batch end V(s_T))
    vals = gold[f"{case}_values"]
    with torch.no_grad():
        v_last = critic(torch.from_numpy(feats[T, :, 0])[None]).item()
    seg_end = done[:, 0].copy()
    seg_end[-1] = 1
    n_seg = int(seg_end.sum())
    boots = np.zeros((n_seg, 8))
    if not done[-1, 0]:
        boots[-1] = np.float32(v_last)
    ret, adv = O.gae(rew[:, :, 0], np.repeat(vals[:, None], 8, 1), boots, seg_end, HP["gamma"], HP["lamb"])
    oa = torch.optim.Adam(actors.parameters(), lr=HP["lr_actor"])
    oc = torch.optim.Adam(critic.parameters(), lr=HP["lr_critic"])
    al, cl = A.update_step(actors, critic, oa, oc, torch.from_numpy(feats[:T]), torch.from_numpy(masks[:T]),
                           torch.from_numpy(acts[:, :, None].copy()), torch.from_numpy(ret[:, :, None]),
                           torch.from_numpy(adv[:, :, None]), gidx, midx, HP["entropy_coef"], HP["max_grad_norm"],
                           dedup=dedup)
    assert np.allclose(al, gold[f"{case}_actor_loss"], rtol=1e-4, atol=1e-6), (al, gold[f"{case}_actor_loss"])
    assert cl == pytest.approx(float(gold[f"{case}_critic_loss"]), rel=1e-4)
    after = _params(actors, critic)
    bad = total = 0
    for k, v in after.items():
        lr = HP["lr_critic"] if k.startswith("critic") else HP["lr_actor"]
        d = ((v - before[k]) / lr).numpy()
        g = gold[f"{case}_delta_{k}"].astype(np.float32)
        err = np.abs(d - g)
        assert err.max() <= 2.0 + 1e-3, k
        bad += int((err > 1e-2).sum())
        total += err.size
    assert bad <= 1e-3 * total, (bad, total)


def test_checkpoint_format_roundtrip(tmp_path):
    """save_model writes the reference's checkpoint dict (a2c.py:733-754); load_model reads
    it with weights_only=True."""
    actors, critic = A.init_networks(seed=5)
    learner = A.VecMultiAgentA2C.__new__(A.VecMultiAgentA2C)
    learner.actors, learner.critic, learner.device = actors, critic, torch.device("cpu")
    learner.obs_dims = dict(zip(spec.AGENTS, A.OBS_DIMS))
    learner.act_dims = dict(zip(spec.AGENTS, A.N_ACTIONS))
    path = tmp_path / "model.pt"
    learner.save_model(str(path))
    ck = torch.load(str(path), weights_only=True)
    assert set(ck) == {"actor_nets", "critic_net", "obs_dims", "act_dims", "global_obs_dim", "possible_agents"}
    assert list(ck["actor_nets"]["agv"]) == ["net.0.weight", "net.0.bias", "net.2.weight", "net.2.bias",
                                             "net.4.weight", "net.4.bias"]
    assert ck["actor_nets"]["agv"]["net.0.weight"].shape == (256, 13)
    assert ck["critic_net"]["net.6.weight"].shape == (1, 128)
    a2, c2 = A.init_networks(seed=6)
    other = A.VecMultiAgentA2C.__new__(A.VecMultiAgentA2C)
    other.actors, other.critic, other.device = a2, c2, torch.device("cpu")
    other.load_model(str(path))
    for k, v in _params(actors, critic).items():
        assert torch.equal(v, _params(a2, c2)[k]), k


def _bare_learner(seed=0):
    actors, critic = A.init_networks(seed=seed)
    learner = A.VecMultiAgentA2C.__new__(A.VecMultiAgentA2C)
    learner.actors, learner.critic, learner.device = actors, critic, torch.device("cpu")
    learner.gidx, learner.midx = A.gather_index("cpu"), A.mask_index("cpu")
    return learner


def test_reference_checkpoint_loads_if_present():
    """The reference's own checkpoints/model.pt through load_model (torch.load(weights_only=
    True) with the numpy scalar / int64 dtype allowlist; a2c.py:733-775): the reference tree is
    absent on the GPU box, where the weights travel as tests/golden/trained_policy.npz."""
    import os
    path = "/root/reference/checkpoints/model.pt"
    if not os.path.exists(path):
        pytest.skip("reference tree not present (GPU box): covered by the trained_policy.npz tests")
    learner = _bare_learner()
    learner.load_model(path)
    ck = A.load_checkpoint(path)
    assert ck["act_dims"] == dict(zip(spec.AGENTS, A.N_ACTIONS)) and ck["global_obs_dim"] == 38
    assert all(type(v) is int for v in ck["act_dims"].values())
    z = np.load(f"{P.GOLDEN}/trained_policy.npz")
    for i, a in enumerate(spec.AGENTS):
        for k, v in ck["actor_nets"][a].items():
            assert torch.equal(learner.actors.actor_state_dict(i)[k], v), (a, k)
            assert np.array_equal(z[f"w_actor.{a}.{k}"], v.numpy()), (a, k)
    for k, v in ck["critic_net"].items():
        assert torch.equal(learner.critic.state_dict()[k], v), k
        assert np.array_equal(z[f"w_critic.{k}"], v.numpy()), k


def test_checkpoint_loader_refuses_other_globals(tmp_path):
    """The allowlist is exactly the numpy scalar + int64 dtype: any other pickled global (here
    a numpy array reconstruction) is refused, never unpickled."""
    path = tmp_path / "bad.pt"
    torch.save({"actor_nets": {}, "x": np.arange(3)}, str(path))
    with pytest.raises(Exception):
        A.load_checkpoint(str(path))


TRAINED = [0, 1, 2, 3, 4, 5, 6, 7]


@pytest.fixture(scope="module")
def trained():
    return np.load(f"{P.GOLDEN}/trained_policy.npz")


@pytest.mark.parametrize("seed", TRAINED)
def test_trained_policy_greedy_matches_reference(trained, seed):
    """The reference's trained weights (npz of checkpoints/model.pt) in the batched policy:
    greedy actions equal the reference's predict(deterministic=True) at every state of its
    test() rollout, values within 1e-5 relative (fp32, per-sample GEMV vs batched GEMM)."""
    learner = _bare_learner()
    learner.load_state_dicts(A.load_npz_weights(f"{P.GOLDEN}/trained_policy.npz"))
    f = torch.from_numpy(trained[f"s{seed}_gstate"].T.copy())          # [38, T]
    m = torch.from_numpy(trained[f"s{seed}_masks"].T.copy())
    with torch.no_grad():
        pm = A.masked_probs(learner.actors(A.actor_inputs(f, learner.gidx)), A.agent_masks(m, learner.midx))
        v = learner.critic(f.t()).view(-1)
    assert np.array_equal(torch.argmax(pm, dim=1).numpy().T, trained[f"s{seed}_actions"])
    assert np.allclose(v.numpy(), trained[f"s{seed}_values"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("seed", [0, 4, 6])
def test_trained_policy_rollout_replays_on_oracle(trained, seed):
    """The reference's test() trajectory under the trained policy: its recorded greedy actions
    replayed through the oracle give the recorded pre-step features, masks and rewards."""
    idx = spec.a2c_feature_index()
    num_orders, steps = int(trained[f"s{seed}_meta"][0]), int(trained[f"s{seed}_meta"][1])
    env = O.OracleEnv()
    r = env.reset(seed=seed, num_orders=num_orders)
    for t in range(steps):
        flat = np.concatenate([r["obs_i32"], r["obs_i8"], r["obs_f32"]]).astype(np.float32)
        assert np.array_equal(flat[idx], trained[f"s{seed}_gstate"][t]), t
        assert np.array_equal(r["masks"], trained[f"s{seed}_masks"][t]), t
        r = env.step(trained[f"s{seed}_actions"][t])
        assert r["rewards"].tobytes() == trained[f"s{seed}_rewards"][t].tobytes(), t


def test_sampler_never_returns_invalid_actions():
    torch.manual_seed(0)
    B = 20000
    probs = torch.softmax(torch.randn(8, 8, B) * 4, dim=1)
    probs[:, :, :100] = 0.0                      # force the uniform fallback on some columns
    masks = (torch.rand(29, B) < 0.5).to(torch.int8)
    for off in A.MASK_OFFS:
        masks[off] = 1
    m = A.agent_masks(masks, A.mask_index("cpu"))
    pm = A.masked_probs(probs, m)
    assert torch.allclose(pm.sum(dim=1), torch.ones(8, B), atol=1e-5)
    for u in (None, torch.zeros(8, 1, B), torch.full((8, 1, B), 1 - 2 ** -24)):
        act = A.sample_categorical(pm, u)
        assert bool((m.gather(1, act.unsqueeze(1)) == 1).all())
        assert bool((pm.gather(1, act.unsqueeze(1)) > 0).all())
    # distribution check on one column
    col = pm[1, :, 500]
    draws = A.sample_categorical(col.view(1, 8, 1).expand(1, 8, 200000).contiguous())
    freq = torch.bincount(draws.view(-1), minlength=8).float() / 200000
    assert torch.allclose(freq, col, atol=5e-3)


def test_log_prob_matches_torch_categorical():
    torch.manual_seed(1)
    p = torch.softmax(torch.randn(8, 8, 300), dim=1)
    a = torch.randint(0, 8, (8, 300))
    ref = torch.distributions.Categorical(probs=p.permute(0, 2, 1)).log_prob(a)
    assert torch.equal(A.categorical_log_prob(p, a), ref)


def test_grouped_update_equals_dense_update():
    """dedup (each network once per distinct input, outputs gathered per sample) gives the
    losses and gradients of the dense update on a batch with many repeated observations: the
    same sums in another order (f32 tolerance)."""
    torch.manual_seed(3)
    T, N = 16, 64
    gen = torch.Generator().manual_seed(5)
    feats = torch.randint(0, 3, (T, A.GLOBAL_DIM, N), generator=gen).float()
    feats[:, 5:9] = torch.randint(0, 40, (T, 4, N), generator=gen).float()   # AGV / pickup: more values
    feats[:, 21] = torch.rand(T, N, generator=gen).round(decimals=1)       # a float progress field
    masks = torch.randint(0, 2, (T, 29, N), generator=gen).to(torch.int8)
    masks[:, A.MASK_OFFS] = 1                                                # IDLE is always valid
    acts = torch.stack([torch.randint(0, n, (T, N), generator=gen) for n in A.N_ACTIONS], 1).to(torch.uint8)
    ret = torch.randn(T, A.NA, N, generator=gen, dtype=torch.float64)
    adv = torch.randn(T, A.NA, N, generator=gen, dtype=torch.float64)
    gidx, midx = A.gather_index("cpu"), A.mask_index("cpu")
    res = []
    for dedup in (False, True):
        actors, critic = A.init_networks(seed=11)
        oa = torch.optim.SGD(actors.parameters(), lr=1.0)
        oc = torch.optim.SGD(critic.parameters(), lr=1.0)
        before = [p.detach().clone() for p in list(actors.parameters()) + list(critic.parameters())]
        al, cl = A.update_step(actors, critic, oa, oc, feats, masks, acts, ret, adv, gidx, midx, 0.01, 1e9,
                               dedup=dedup)
        after = [p.detach().clone() for p in list(actors.parameters()) + list(critic.parameters())]
        res.append((al, cl, [b - a for a, b in zip(after, before)]))
    (al0, cl0, g0), (al1, cl1, g1) = res
    assert np.allclose(al0, al1, rtol=1e-5, atol=1e-6)
    assert cl1 == pytest.approx(cl0, rel=1e-5)
    for a, b in zip(g0, g1):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-6)
    # the grouping itself: repeated columns share an index, a collision is detected
    x = feats.permute(1, 0, 2).reshape(A.GLOBAL_DIM, -1)[:7]
    g = A.group_columns(x)
    assert torch.equal(x[:, g.rep[0]], x) and g.U[0] < x.shape[1]
    assert torch.equal(x[:, g.first[0]][:, g.inv[0]], x)
    y = torch.randn(1, 3, g.U[0], dtype=torch.float32, requires_grad=True)
    w = torch.randn(1, 3, x.shape[1])
    (g.gather(y) * w).sum().backward()
    ref = torch.zeros(3, g.U[0]).index_add_(1, g.inv[0], w[0])
    assert torch.allclose(y.grad[0], ref, rtol=1e-5, atol=1e-5)
    assert A.group_columns(x, torch.zeros(x.shape[1], dtype=torch.int64)) is None


def test_policy_weight_packing_planes_and_lane_order():
    """pack_mfma (the fused policy kernel's weight layout, include/fjsp.h): three bf16 planes
    whose sum is the f32 weight within 2^-24 relative, in the 32x32x16 MFMA A-operand lane order
    (t, kb, p, l, j) = plane p of W[32 t + (l & 31)][16 kb + 8 (l >> 5) + j]."""
    g = torch.Generator().manual_seed(5)
    W = torch.randn(64, 48, generator=g) * torch.logspace(-3, 2, 48)[None, :]
    hi, mid, lo = A.split_bf16x3(W)
    back = hi.double() + mid.double() + lo.double()
    assert float(((back - W.double()).abs() / W.double().abs()).max()) <= 2.0 ** -24
    Pk = A.pack_mfma(W).view(torch.bfloat16).reshape(2, 3, 3, 64, 8)   # t, kb, p, l, j
    planes = (hi, mid, lo)
    for t, kb, p, l, j in [(0, 0, 0, 0, 0), (1, 2, 1, 37, 5), (1, 1, 2, 63, 7), (0, 2, 0, 31, 3)]:
        r, k = 32 * t + (l & 31), 16 * kb + 8 * (l >> 5) + j
        assert Pk[t, kb, p, l, j].item() == planes[p][r, k].item()
    a, c = A.pack_policy_weights(*A.init_networks(seed=0))
    assert a.numel() == 8 * A.nat.POLICY_ACTOR_FLOATS and c.numel() == A.nat.POLICY_CRITIC_FLOATS
