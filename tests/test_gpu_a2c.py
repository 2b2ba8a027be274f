"""End-to-end batched A2C on the GPU (a2c_vec.VecMultiAgentA2C over FJSPVecEnv) against the
reference's MultiAgentA2C.learn fixtures (tests/golden/gen_a2c_golden.py), plus masked sampling
and multi-env sanity.  Tolerances as in tests/test_a2c_learner.py (fp32 network math)."""
import importlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import parity_util as P  # noqa: E402


@pytest.fixture(scope="module")
def M():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from tests import gpu_util  # noqa: F401
    return {"A": importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec"),
            "V": importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env"),
            "spec": importlib.import_module("multi-agent-rl-for-fjsp_amd.spec")}


def _deltas(A, spec, learner, before):
    out = {}
    for i, a in enumerate(spec.AGENTS):
        for k, v in learner.actors.actor_state_dict(i).items():
            out[f"actor.{a}.{k}"] = ((v - before[f"actor.{a}.{k}"]) / 3e-4).numpy()
    for k, v in learner.critic.state_dict().items():
        out[f"critic.{k}"] = ((v.detach().cpu() - before[f"critic.{k}"]) / 1e-3).numpy()
    return out


def _snapshot(spec, learner):
    out = {}
    for i, a in enumerate(spec.AGENTS):
        for k, v in learner.actors.actor_state_dict(i).items():
            out[f"actor.{a}.{k}"] = v
    for k, v in learner.critic.state_dict().items():
        out[f"critic.{k}"] = v.detach().cpu().clone()
    return out


@pytest.mark.parametrize("case", ["greedy", "replay"])
def test_learn_matches_reference(M, case):
    A, V, spec = M["A"], M["V"], M["spec"]
    g = np.load(f"{P.GOLDEN}/a2c_golden.npz")
    env = V.FJSPVecEnv(1)
    learner = A.VecMultiAgentA2C(env, batch_size=256, seed=0)
    before = _snapshot(spec, learner)
    action_fn = None
    if case == "replay":
        def action_fn(t, masks):
            return torch.from_numpy(O.actions(99, 0, t, masks[:, 0].cpu().numpy()).astype(np.int64))[:, None]
    learner.learn(256, num_orders=25, seeds=[0], deterministic=(case == "greedy"), action_fn=action_fn)
    b = learner._bufs
    assert np.array_equal(b["actions"][:, :, 0].cpu().numpy(), g[f"{case}_actions"])
    assert np.allclose(b["values"][:256, 0].cpu().numpy(), g[f"{case}_values"], atol=1e-5, rtol=1e-5)
    al = [learner.actor_loss_history[a][0] for a in spec.AGENTS]
    assert np.allclose(al, g[f"{case}_actor_loss"], rtol=1e-4, atol=1e-6)
    assert learner.critic_loss_history[0] == pytest.approx(float(g[f"{case}_critic_loss"]), rel=1e-4)
    bad = total = 0
    for k, d in _deltas(A, spec, learner, before).items():
        err = np.abs(d - g[f"{case}_delta_{k}"].astype(np.float32))
        assert err.max() <= 2.0 + 1e-3, k
        bad += int((err > 1e-2).sum())
        total += err.size
    assert bad <= 1e-3 * total, (bad, total)


def test_sampling_respects_masks_and_trains(M):
    A, V = M["A"], M["V"]
    n = 512
    env = V.FJSPVecEnv(n)
    learner = A.VecMultiAgentA2C(env, batch_size=64, seed=1)
    learner.learn(2 * 64 * n, num_orders=25, seeds=torch.arange(n))
    b = learner._bufs
    # step t acted on masks[t]; masks[0] was replaced by roll_over() after the last update
    acts = b["actions"][1:].long()                                   # [T-1, 8, N]
    masks = b["masks"][1:64]
    for a in range(8):
        chosen = masks[:, A.MASK_OFFS[a]:A.MASK_OFFS[a] + A.N_ACTIONS[a], :].gather(1, acts[:, a:a + 1, :])
        assert bool((chosen == 1).all()), a
    assert len(learner.critic_loss_history) == 2
    assert all(np.isfinite(learner.critic_loss_history))
    assert int(b["status"].bitwise_and(1).sum()) == 0
    f, m = env.pack_a2c()
    assert torch.equal(f, b["feats"][64]) and torch.equal(m, b["masks"][64])


def test_sampled_rollout_features_match_oracle(M):
    """One sampled batch on 256 envs: the features / masks / rewards the learner consumed equal
    the oracle's replay of the sampled actions."""
    A, V, spec = M["A"], M["V"], M["spec"]
    n, T = 256, 96
    env = V.FJSPVecEnv(n)
    learner = A.VecMultiAgentA2C(env, batch_size=T, seed=2)
    learner.reset(seeds=torch.arange(n) + 40, num_orders=25)
    learner.collect()
    b = learner._bufs
    idx = spec.a2c_feature_index()
    acts = b["actions"].cpu().numpy()                                # [T, 8, N]
    feats, masks, rew = b["feats"].cpu().numpy(), b["masks"].cpu().numpy(), b["rewards"].cpu().numpy()
    for e in (0, 77, 255):
        o = O.OracleEnv()
        r = o.reset(seed=40 + e, num_orders=25)
        for t in range(T):
            flat = np.concatenate([r["obs_i32"], r["obs_i8"], r["obs_f32"]]).astype(np.float32)
            assert P.bits_equal(feats[t, :, e], flat[idx]), (e, t)
            assert P.bits_equal(masks[t, :, e], r["masks"]), (e, t)
            r = o.step(acts[t, :, e])
            assert P.bits_equal(rew[t, :, e], r["rewards"]), (e, t)
            if r["term"] or r["trunc"]:
                r = o.reset(num_orders=25)


def test_graph_replay_equals_eager(M):
    """The hipGraph-captured collect phase computes exactly what the eager loop computes."""
    A, V = M["A"], M["V"]
    n, T = 256, 32
    runs = []
    for use_graph in (False, True):
        env = V.FJSPVecEnv(n)
        learner = A.VecMultiAgentA2C(env, batch_size=T, seed=4, use_graph=use_graph)
        learner.learn(3 * T * n, num_orders=25, seeds=torch.arange(n), deterministic=True)
        b = learner._bufs
        runs.append((learner.critic_loss_history, [learner.actor_loss_history[a] for a in M["spec"].AGENTS],
                     b["actions"].cpu(), b["feats"].cpu(), b["rewards"].cpu()))
    assert runs[1][0] == runs[0][0] and runs[1][1] == runs[0][1]
    for i in (2, 3, 4):
        assert torch.equal(runs[0][i], runs[1][i])


@pytest.mark.parametrize("n,T,det,graph,groups", [(1000, 210, False, True, 2), (4096, 256, False, True, 4),
                                                  (4096, 256, False, True, 1), (130, 70, True, False, 2),
                                                  (64, 230, False, True, 2)])
def test_policy_step_launch_equals_two_launches(M, n, T, det, graph, groups):
    """fjsp_a2c_policy_step (policy + env step in one launch, the step of each 64-env tile run by
    its last actor workgroup after the write-through action hand-off) == fjsp_a2c_policy then
    fjsp_step: every byte of the rollout slab over three batches (eager, captured, replayed),
    partial tiles, greedy and sampled actions, across auto-resets; the env groups of the collect
    on concurrent streams (collect_groups) change nothing."""
    A, V = M["A"], M["V"]
    keys = ("feats", "masks", "actions", "values", "rewards", "term", "trunc", "status")
    runs = []
    for fused in (False, True):
        env = V.FJSPVecEnv(n)
        L = A.VecMultiAgentA2C(env, batch_size=T, seed=21, use_graph=graph)
        L.fused_step = fused
        L.collect_groups = groups
        L.reset(seeds=torch.arange(n) + 7, num_orders=25)
        out = []
        for _ in range(3):
            L.collect(deterministic=det)
            out.append({k: L._bufs[k].clone() for k in keys})
            L.roll_over()
        assert env.last_kernel() == "k_policy_step" if fused else env.last_kernel().startswith("k_step")
        runs.append(out)
    for b in range(3):
        for k in keys:
            assert torch.equal(runs[0][b][k], runs[1][b][k]), (b, k)
    ends = sum(int((r["term"] | r["trunc"]).sum()) for r in runs[1])
    assert ends >= n                                    # every env crossed an auto-reset


@pytest.mark.parametrize("var,values", [("policy_dedup", (0, 1)), ("policy_split", (0, 1)),
                                        ("policy_xmap", (0, 1, 2, 3))])
@pytest.mark.parametrize("n,init", [(4096, "random"), (1000, "trained")])
def test_policy_launch_variants_are_bit_identical(M, n, init, var, values):
    """The policy launch's work splits change which workgroup computes what, never a value:
    the station agents' MLP once per distinct input of a 64-env tile on one 32-env column tile
    (policy_dedup, on by default) == the MLP on every env; the pickup station's and the AGV's
    tiles as two 32-env workgroups each (policy_split, on by default) == one 64-env workgroup;
    the three XCD-aware workgroup orders (policy_xmap 1-3, which run without the split) == the
    default order.  Library-wide options (fjsp_set_option(NULL, ...)).  Every byte of the rollout
    slabs over two batches with an update between them (the second batch acts with updated
    weights), partial tiles, random-init and trained networks."""
    import os
    A, V = M["A"], M["V"]
    nat = A.nat
    keys = ("feats", "masks", "actions", "values", "rewards", "term", "trunc", "status")
    default = {"policy_dedup": 1, "policy_split": 1, "policy_xmap": 0}[var]

    def run(v):
        nat.check(nat.lib().fjsp_set_option(None, var.encode(), v))
        try:
            L = A.VecMultiAgentA2C(V.FJSPVecEnv(n), batch_size=64, seed=4)
            if init == "trained":
                L.load_state_dicts(A.load_npz_weights(os.path.join(os.path.dirname(__file__), "golden",
                                                                   "trained_policy.npz")))
            L.reset(seeds=torch.arange(n) + 3, num_orders=25)
            out = []
            for _ in range(2):
                L.collect()
                out.append({k: L._bufs[k].clone() for k in keys})
                L.update()
                L.roll_over()
            return out
        finally:
            nat.check(nat.lib().fjsp_set_option(None, var.encode(), default))
    runs = [run(v) for v in values]
    for r in runs[1:]:
        for b in range(2):
            for k in keys:
                assert torch.equal(runs[0][b][k], r[b][k]), (b, k)


def test_collect_graphs_interleaved_with_allocations(M):
    """Two learners' captured collects (each graph in its own private pool) replayed in turn, with
    an update, a recapture (deterministic toggled) and allocation churn between the replays, equal
    their eager twins byte for byte: nothing allocated after a capture may land in a live graph's
    memory (the aliasing that made r04's shared-pool update graphs diverge)."""
    A, V = M["A"], M["V"]
    n, T = 320, 24
    keys = ("feats", "masks", "actions", "values", "rewards", "term", "trunc", "status")
    L = {}
    for name, seed in (("a", 5), ("b", 6)):
        for graph in (True, False):
            x = A.VecMultiAgentA2C(V.FJSPVecEnv(n), batch_size=T, seed=seed, use_graph=graph)
            x.reset(seeds=torch.arange(n) + seed, num_orders=25)
            L[name, graph] = x
    junk = []
    for it in range(5):
        det = it == 3                                   # batch 3 recaptures (deterministic), 4 again
        for name in ("a", "b"):
            for graph in (True, False):
                L[name, graph].collect(deterministic=det)
            junk.append(torch.randn(1 << 20, device="cuda") * it)   # churn between the replays
            if len(junk) > 3:
                junk.pop(0)
            for k in keys:
                assert torch.equal(L[name, True]._bufs[k], L[name, False]._bufs[k]), (it, name, k)
            for graph in (True, False):
                L[name, graph].update()
                L[name, graph].roll_over()
        torch.cuda.empty_cache()


def test_eager_policy_graph_rekeys_each_batch(M):
    """The PyTorch policy path (fused_policy=False) captured into the collect graph reads the
    draw key from the device: every replay draws new actions, and each batch equals the eager
    loop's (same weights: no update between the batches)."""
    A, V = M["A"], M["V"]
    n, T = 256, 16
    runs = []
    for use_graph in (False, True):
        env = V.FJSPVecEnv(n)
        L = A.VecMultiAgentA2C(env, batch_size=T, seed=8, use_graph=use_graph, fused_policy=False)
        L.reset(seeds=torch.arange(n), num_orders=25)
        acts = []
        for _ in range(4):
            L.collect()
            acts.append(L._bufs["actions"].clone())
            L.roll_over()
        assert (L._graph is not None) == use_graph
        runs.append(acts)
    eager, graph = runs
    for b in range(4):
        assert torch.equal(eager[b], graph[b]), b
    # replays of one captured graph draw new actions (a frozen key would repeat the AGV's
    # choices wherever the observation repeats; here whole batches would coincide only then)
    assert not torch.equal(graph[2], graph[3])
    L._rng.fill_(12345)
    a0 = L.policy(L._bufs["feats"][0], L._bufs["masks"][0], t=0)[0]
    L._rng.fill_(12346)
    a1 = L.policy(L._bufs["feats"][0], L._bufs["masks"][0], t=0)[0]
    assert not torch.equal(a0, a1)                      # the device key reaches the eager draw


def test_fused_policy_kernel_matches_torch_policy(M):
    """fjsp_a2c_policy (one MFMA kernel per step) == the PyTorch policy path: masked
    probabilities and values within 1e-5, greedy actions equal (up to near-ties), sampled
    actions valid and distributed like the probabilities."""
    A, V = M["A"], M["V"]
    n = 1000                                                          # not a multiple of 64
    env = V.FJSPVecEnv(n)
    learner = A.VecMultiAgentA2C(env, batch_size=8, seed=3, use_graph=False)
    learner.learn(2 * 8 * n, num_orders=25, seeds=torch.arange(n))   # two updates: trained weights
    feats, masks = env.pack_a2c()
    act_t, pm_t, v_t = learner.policy(feats, masks, deterministic=True)
    act = torch.zeros(8, n, dtype=torch.uint8, device=env.device)
    val = torch.zeros(n, dtype=torch.float32, device=env.device)
    probs = torch.zeros(8, 8, n, dtype=torch.float32, device=env.device)
    learner.policy_fused(feats, masks, 0, True, act, val, probs)
    torch.cuda.synchronize()
    assert torch.allclose(probs, pm_t, atol=1e-5), float((probs - pm_t).abs().max())
    assert torch.allclose(val, v_t, atol=1e-5, rtol=1e-5), float((val - v_t).abs().max())
    top2 = torch.topk(pm_t, 2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-5
    assert bool((act.long() == act_t)[clear].all())
    # sampling: valid actions, frequencies ~ probabilities
    ma = A.agent_masks(masks, learner.midx)
    counts = torch.zeros(8, 8, n, device=env.device)
    R = 400
    for r in range(R):
        learner._rng.fill_(1000 + r)
        learner.policy_fused(feats, masks, 0, False, act, val)
        assert bool((ma.gather(1, act.long().unsqueeze(1)) == 1).all())
        counts.scatter_add_(1, act.long().unsqueeze(1), torch.ones(8, 1, n, device=env.device))
    freq = counts / R
    assert float((freq - pm_t).abs().mean()) < 0.01


def test_fused_policy_error_is_f32_level(M):
    """The fused kernel computes its layers with f32 operands split into three bf16 planes on the
    bf16 matrix cores (csrc/fjsp_policy.hip): its error against a float64 evaluation of the same
    networks is at the level of PyTorch's f32 policy path (bounded here by 2x that path's error
    plus 1e-7), and its greedy actions equal the float64 argmax wherever the top-2 margin
    exceeds 1e-5 (profiles/r03/policy_split/accuracy_*.json: 4 096 envs x 16 steps)."""
    import copy
    A, V = M["A"], M["V"]
    n = 1000
    env = V.FJSPVecEnv(n)
    learner = A.VecMultiAgentA2C(env, batch_size=8, seed=6, use_graph=False)
    learner.learn(2 * 8 * n, num_orders=25, seeds=torch.arange(n))
    feats, masks = env.pack_a2c()
    act64, crit64 = copy.deepcopy(learner.actors).double(), copy.deepcopy(learner.critic).double()
    with torch.no_grad():
        pm64 = A.masked_probs(act64(A.actor_inputs(feats.double(), learner.gidx)), A.agent_masks(masks, learner.midx))
        v64 = crit64(feats.double().t()).view(-1)
        _, pm32, v32 = learner.policy(feats, masks, deterministic=True)
    act = torch.zeros(8, n, dtype=torch.uint8, device=env.device)
    val = torch.zeros(n, dtype=torch.float32, device=env.device)
    probs = torch.zeros(8, 8, n, dtype=torch.float32, device=env.device)
    learner.policy_fused(feats, masks, 0, True, act, val, probs)
    torch.cuda.synchronize()
    ep, ep32 = float((probs.double() - pm64).abs().max()), float((pm32.double() - pm64).abs().max())
    ev, ev32 = float((val.double() - v64).abs().max()), float((v32.double() - v64).abs().max())
    assert ep <= 2 * ep32 + 1e-7, (ep, ep32)
    assert ev <= 2 * ev32 + 1e-7, (ev, ev32)
    top2 = torch.topk(pm64, 2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-5
    assert bool((act.long() == torch.argmax(pm64, dim=1))[clear].all())


def test_eager_and_fused_draws_share_the_counter_hash(M):
    """Both policy paths draw with the (seed, global env id, step, agent) counter hash: with the
    same key the sampled actions agree except where the probabilities differ by rounding right
    at a CDF step; a shard's draws (env_id_base) are the big handle's for the same global ids."""
    A, V = M["A"], M["V"]
    n = 512
    env = V.FJSPVecEnv(n, env_id_base=3 * n)
    learner = A.VecMultiAgentA2C(env, batch_size=8, seed=21, use_graph=False)
    learner.reset(num_orders=25)
    feats, masks = env.pack_a2c()
    act = torch.zeros(8, n, dtype=torch.uint8, device=env.device)
    val = torch.zeros(n, dtype=torch.float32, device=env.device)
    learner._rng.fill_(learner._rng_host)
    learner.policy_fused(feats, masks, 7, False, act, val)
    act_t = learner.policy(feats, masks, deterministic=False, t=7)[0]
    torch.cuda.synchronize()
    assert float((act.long() == act_t).float().mean()) > 0.999
    u_shard = A.counter_uniform(learner._rng_host, torch.arange(3 * n, 4 * n), 7, "cpu")
    u_big = A.counter_uniform(learner._rng_host, torch.arange(0, 4 * n), 7, "cpu")
    assert torch.equal(u_shard, u_big[..., 3 * n:])


def test_a2c_4096_envs_grouped_update(M):
    """A 4096-env x 64-step batch (BASELINE config 4's env count): sampled actions respect the
    masks, three sampled envs replay on the oracle, the group-key kernel equals the host hash,
    and the grouped update (dedup: each network once per distinct input) moves every parameter
    as the dense update does, with finite losses."""
    A, V, spec = M["A"], M["V"], M["spec"]
    n, T = 4096, 64
    env = V.FJSPVecEnv(n)
    learner = A.VecMultiAgentA2C(env, batch_size=T, seed=4)
    learner.reset(seeds=torch.arange(n) + 7, num_orders=25)
    learner.collect()
    b = learner._bufs
    acts = b["actions"].long()
    for a in range(8):
        chosen = b["masks"][:T, A.MASK_OFFS[a]:A.MASK_OFFS[a] + A.N_ACTIONS[a], :].gather(1, acts[:, a:a + 1, :])
        assert bool((chosen == 1).all()), a
    idx = spec.a2c_feature_index()
    feats, masks, rew = b["feats"].cpu().numpy(), b["masks"].cpu().numpy(), b["rewards"].cpu().numpy()
    an = acts.cpu().numpy()
    for e in (0, 2049, 4095):
        o = O.OracleEnv()
        r = o.reset(seed=7 + e, num_orders=25)
        for t in range(T):
            flat = np.concatenate([r["obs_i32"], r["obs_i8"], r["obs_f32"]]).astype(np.float32)
            assert P.bits_equal(feats[t, :, e], flat[idx]), (e, t)
            assert P.bits_equal(masks[t, :, e], r["masks"]), (e, t)
            r = o.step(an[t, :, e])
            assert P.bits_equal(rew[t, :, e], r["rewards"]), (e, t)
            if r["term"] or r["trunc"]:
                r = o.reset(num_orders=25)
    keys = A.group_keys(b["feats"][:T])
    assert torch.equal(keys.cpu(), A.group_keys(b["feats"][:T].cpu()))
    ret, adv = learner.advantages()
    res = []
    for dedup in (False, True):
        actors, critic = A.init_networks(seed=9, device="cuda")
        oa = torch.optim.SGD(actors.parameters(), lr=1.0)
        oc = torch.optim.SGD(critic.parameters(), lr=1.0)
        before = [p.detach().clone() for p in list(actors.parameters()) + list(critic.parameters())]
        al, cl = A.update_step(actors, critic, oa, oc, b["feats"][:T], b["masks"][:T], b["actions"], ret, adv,
                               learner.gidx, learner.midx, 0.01, 1e9, dedup=dedup)
        assert np.all(np.isfinite(al)) and np.isfinite(cl)
        res.append((al, cl, [(bb - p.detach()) for bb, p in zip(before, list(actors.parameters()) +
                                                                 list(critic.parameters()))]))
    (al0, cl0, g0), (al1, cl1, g1) = res
    assert np.allclose(al0, al1, rtol=1e-4, atol=1e-6)
    assert cl1 == pytest.approx(cl0, rel=1e-4)
    for x, y in zip(g0, g1):
        scale = float(x.abs().max()) + 1e-12
        assert float((x - y).abs().max()) <= 1e-3 * scale


def test_group_verify_kernel_flags_collisions(M):
    """fjsp_a2c_group_verify accepts a true grouping (equal to the torch comparison) and flags
    a forged one: an actor representative or a global-state representative whose inputs
    differ from the sample's (what a hash collision would produce)."""
    A = M["A"]
    T, n = 3, 700
    g = torch.Generator().manual_seed(5)
    base = torch.randint(0, 4, (T, 38, n), generator=g).float()
    base[:, :, n // 2:] = base[:, :, :n - n // 2]              # duplicated columns
    f = base.cuda()
    keys = A.group_keys(f)
    ga, gc = A.RowGroups(keys[:A.NA]), A.RowGroups(keys[A.NA:])
    x = A.actor_inputs(f, A.gather_index(f.device))
    gt = f.permute(1, 0, 2).reshape(A.GLOBAL_DIM, -1)
    assert A.group_verify(f, ga, gc)
    assert bool((torch.gather(x, 2, ga.rep[:, None, :].expand_as(x)) == x).all())
    S = T * n
    s = 1234
    other = int((gt[:, s + 1:] != gt[:, s:s + 1]).any(0).nonzero()[0]) + s + 1   # a column unlike s
    bad_c = _copy(gc)
    bad_c.rep = gc.rep.clone()
    bad_c.rep[0, s] = other
    assert not A.group_verify(f, ga, bad_c)
    for a in (0, 1, 7):
        cols = A.gather_index(f.device)[a, :A.OBS_DIMS[a]]
        o = int((gt[cols, :] != gt[cols, s:s + 1]).any(0).nonzero()[0])
        bad_a = _copy(ga)
        bad_a.rep = ga.rep.clone()
        bad_a.rep[a, s] = o
        assert not A.group_verify(f, bad_a, gc), a
    assert S == gt.shape[1]


def _copy(g):
    """A shallow copy of RowGroups g (its rep replaced by the caller)."""
    c = type(g).__new__(type(g))
    c.__dict__.update(g.__dict__)
    return c


@pytest.mark.parametrize("rows", [65536, 70001])
def test_critic_splitk_relu_backward(M, rows):
    """The critic MLP over a long batch through mlp_forward (split-K weight gradients, ReLU in
    the GEMM epilogue, fjsp_a2c_relu_bias_grad for ReLU backward + bias gradient) equals
    nn.Sequential autograd in fp32 (relative 1e-5 on outputs, 1e-4 on gradients)."""
    A = M["A"]
    torch.manual_seed(3)
    critic = A.CriticNet(A.GLOBAL_DIM).cuda()
    x = torch.randn(A.GLOBAL_DIM, rows, device="cuda").t()
    w = torch.randn(rows, 1, device="cuda")
    y1 = A.mlp_forward(critic.net, x)
    (y1 * w).sum().backward()
    g1 = [p.grad.clone() for p in critic.parameters()]
    critic.zero_grad(set_to_none=True)
    y2 = critic.net(x)
    (y2 * w).sum().backward()
    assert float((y1 - y2).detach().abs().max()) <= 1e-5 * float(y2.detach().abs().max())
    for a, p in zip(g1, critic.parameters()):
        assert float((a - p.grad).abs().max()) <= 1e-4 * float(p.grad.abs().max())


def test_fused_policy_forced_tiles(M):
    """A 64-env tile in which an agent has exactly one valid action in every env skips the
    actor's MLP in fjsp_a2c_policy: its actions are that action (greedy and sampled) and its
    probabilities exactly one-hot, as the full path gives (masked renormalisation p / p); a tile
    with one unforced env, and the critic's values, match the PyTorch policy path."""
    A, V = M["A"], M["V"]
    n = 1000
    env = V.FJSPVecEnv(n)
    learner = A.VecMultiAgentA2C(env, batch_size=8, seed=5, use_graph=False)
    learner.reset(seeds=torch.arange(n), num_orders=25)
    g = torch.Generator(device=env.device).manual_seed(11)
    feats = torch.randint(0, 6, (A.GLOBAL_DIM, n), device=env.device, generator=g).float()
    masks = (torch.rand(29, n, device=env.device, generator=g) < 0.6).to(torch.int8)
    for a in range(8):
        o = A.MASK_OFFS[a]
        masks[o, :] = 1                                             # at least one valid action
    forced_envs = torch.arange(0, 128, device=env.device)
    for a in range(2, 8):                                            # the station agents
        o = A.MASK_OFFS[a]
        j = (forced_envs + a) % 3
        masks[o:o + 3, :128] = 0
        masks[o + j, forced_envs] = 1
        masks[o:o + 3, 100] = 1                                      # tile 1 has one unforced env
    act_t, pm_t, v_t = learner.policy(feats, masks, deterministic=True)
    act = torch.zeros(8, n, dtype=torch.uint8, device=env.device)
    val = torch.zeros(n, dtype=torch.float32, device=env.device)
    probs = torch.zeros(8, 8, n, dtype=torch.float32, device=env.device)
    learner.policy_fused(feats, masks, 0, True, act, val, probs)
    torch.cuda.synchronize()
    assert torch.allclose(probs, pm_t, atol=1e-5) and torch.allclose(val, v_t, atol=1e-5, rtol=1e-5)
    for a in range(2, 8):
        j = ((forced_envs + a) % 3)[:64]
        onehot = torch.nn.functional.one_hot(j, 8).float().t()
        assert torch.equal(probs[a][:, :64], onehot), a                # skipped tile: exact one-hot
        assert torch.equal(act[a, :64].long(), j), a
        assert torch.equal(probs[a][:, 64:128][:, torch.arange(64) != 36],
                           torch.nn.functional.one_hot(((forced_envs + a) % 3)[64:], 8).float().t()
                           [:, torch.arange(64) != 36]), a             # full path, forced envs
    for r in range(5):
        learner._rng.fill_(77 + r)
        learner.policy_fused(feats, masks, r, False, act, val)
        for a in range(2, 8):
            assert torch.equal(act[a, :64].long(), ((forced_envs + a) % 3)[:64]), a


def test_a2c_config4_full_batch(M):
    """BASELINE config 4 at its size: 4 096 envs x one 256-step batch (train.py --batch_size 256,
    num_orders 25).  Sampled actions respect the masks, every 8th env (512, both env groups of the
    collect, every workgroup position) replays on the oracle over the whole batch (features,
    masks, rewards bit-exact), and the grouped update's gradients equal the
    dense update's to 1e-4 relative per parameter tensor (the same sum of ~10^6 f32 terms per
    weight in another order: f64 run sums over groups against f32 GEMM accumulation)."""
    A, V, spec = M["A"], M["V"], M["spec"]
    n, T = 4096, 256
    env = V.FJSPVecEnv(n)
    learner = A.VecMultiAgentA2C(env, batch_size=T, seed=12)
    learner.reset(seeds=torch.arange(n) + 500, num_orders=25)
    learner.collect()
    b = learner._bufs
    acts = b["actions"].long()
    for a in range(8):
        chosen = b["masks"][:T, A.MASK_OFFS[a]:A.MASK_OFFS[a] + A.N_ACTIONS[a], :].gather(1, acts[:, a:a + 1, :])
        assert bool((chosen == 1).all()), a
    idx = spec.a2c_feature_index()
    feats, masks, rew = b["feats"].cpu().numpy(), b["masks"].cpu().numpy(), b["rewards"].cpu().numpy()
    an = acts.cpu().numpy()
    for e in list(range(1, n, 8)) + [4094]:
        o = O.OracleEnv()
        r = o.reset(seed=500 + e, num_orders=25)
        for t in range(T):
            flat = np.concatenate([r["obs_i32"], r["obs_i8"], r["obs_f32"]]).astype(np.float32)
            assert P.bits_equal(feats[t, :, e], flat[idx]), (e, t)
            assert P.bits_equal(masks[t, :, e], r["masks"]), (e, t)
            r = o.step(an[t, :, e])
            assert P.bits_equal(rew[t, :, e], r["rewards"]), (e, t)
            if r["term"] or r["trunc"]:
                r = o.reset(num_orders=25)
    ret, adv = learner.advantages()
    grads, losses = [], []
    for dedup in (False, True):
        actors, critic = A.init_networks(seed=13, device="cuda")
        oa = torch.optim.Adam(actors.parameters(), lr=3e-4)
        oc = torch.optim.Adam(critic.parameters(), lr=1e-3)
        losses.append(A.update_step(actors, critic, oa, oc, b["feats"][:T], b["masks"][:T], b["actions"], ret, adv,
                                    learner.gidx, learner.midx, 0.01, 0.5, dedup=dedup,
                                    grad_probe=lambda g: grads.append(g.cpu())))
    P.assert_grads_close(grads[1], grads[0], rel=1e-4)
    # the loss VALUES of both updates against the reference's formulas (a2c.py:694-731) restated
    # in float64 over the whole 4 096 x 256 batch, from the same initial weights
    ref_al, ref_cl = _reference_losses_f64(A, spec, b["feats"][:T], b["masks"][:T], b["actions"], ret, adv, 13)
    for al, cl in losses:
        for a in range(8):
            assert abs(al[a] - ref_al[a]) <= 1e-5 * abs(ref_al[a]) + 1e-7, (a, al[a], ref_al[a])
        assert abs(cl - ref_cl) <= 1e-5 * abs(ref_cl), (cl, ref_cl)
    # test_agents_configs-style exclusion count: no env of this batch left the closed form
    assert int((b["status"][:T] & 1).sum()) == 0


def _reference_losses_f64(A, spec, feats, masks, actions, ret, adv, seed, entropy_coef=0.01):
    """MultiAgentA2C._update's loss values (a2c.py:647-731) over every transition of a [T, ., N]
    batch, in float64 with plain torch ops (networks.py layouts rebuilt from the reference-format
    state dicts of init_networks(seed)):
      actor a: calc_actor_loss(logprob, adv) - entropy_coef * _calculate_entropy, where logprob is
        log of the action's probability under the masked, renormalised distribution (predict,
        a2c.py:208-238; uniform over the valid actions when the masked sum is 0), the advantages
        are normalised with their float32 mean and unbiased std (+1e-8), and the entropy is the
        mean over samples of -sum p log(p + 1e-10) of the UNMASKED probabilities;
      critic: F.mse_loss over every agent's (value, return) pair = mean over 8 T N of (V - R)^2."""
    import torch.nn as nn
    T, _, N = feats.shape
    S = T * N
    actors, critic = A.init_networks(seed=seed, device="cpu")
    x = feats.permute(0, 2, 1).reshape(S, A.GLOBAL_DIM).double()                 # [S, 38]
    m = masks.permute(0, 2, 1).reshape(S, A.MASK_DIM).double()
    act = actions.permute(0, 2, 1).reshape(S, 8).long()
    R = ret.permute(0, 2, 1).reshape(S, 8)
    adv32 = adv.float().permute(0, 2, 1).reshape(S, 8)
    al = []
    for a in range(8):
        sd = actors.actor_state_dict(a)
        d, k = spec.A2C_OBS_DIMS[spec.AGENTS[a]], spec.N_ACTIONS[a]
        net = nn.Sequential(nn.Linear(d, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, k),
                            nn.Softmax(dim=-1)).double().cuda()
        net.load_state_dict({kk.replace("net.", ""): v.double() for kk, v in sd.items()})
        with torch.no_grad():
            p = net(x[:, A.OBS_OFFS[a]:A.OBS_OFFS[a] + d])                               # [S, k]
        mk = m[:, A.MASK_OFFS[a]:A.MASK_OFFS[a] + k]
        pm = p * mk
        ssum = pm.sum(1, keepdim=True)
        pm = torch.where(ssum > 0, pm / ssum.clamp_min(1e-300), mk / mk.sum(1, keepdim=True))
        logp = torch.log(pm.gather(1, act[:, a:a + 1]).reshape(-1))
        v = adv32[:, a]
        vn = ((v - v.mean()) / (v.std() + 1e-8)).double()                               # float32 statistics
        ent = (-(p * torch.log(p + 1e-10)).sum(1)).mean()
        al.append(float(-(vn * logp).mean() - entropy_coef * ent))
    cnet = critic.net.double().cuda()
    with torch.no_grad():
        V = cnet(x).reshape(-1)                                                        # [S]
    cl = float(((V[:, None] - R.float().double()) ** 2).mean())
    return al, cl


def test_fused_critic_forward_backward_matches_torch(M):
    """The grouped update's critic (a2c_vec._CriticGrouped: fjsp_a2c_critic_forward, then the
    value-head / ReLU-bias kernels and split-K weight gradients) against a float64 evaluation of
    the same network, beside the PyTorch-GEMM path (mlp_forward): values at most 3x that f32
    path's error (+1e-7 relative), every parameter gradient within max(3x its error, 3e-3)
    relative.  Both f32 paths flip a ReLU unit here and there whose pre-activation is within
    rounding of 0 (scripts/diag_critic_fused.py: one per layer of 70 001 x 256 for either path, the
    activations themselves within 7e-7 of float64), and one flipped unit of one sample moves a
    weight gradient summed over 70 001 samples by ~3e-4 relative; a layout or indexing error
    moves it by O(1)."""
    import copy
    A = M["A"]
    torch.manual_seed(3)
    _, critic = A.init_networks(seed=1, device="cuda")
    U = 70001
    xT = (torch.rand(38, U, device="cuda") * torch.randint(0, 30, (38, 1), device="cuda")).float()
    w = torch.randn(U, device="cuda")
    c64 = copy.deepcopy(critic).double()
    v64 = c64.net(xT.double().t()).reshape(-1)
    (v64 * w.double()).sum().backward()
    g64 = [p.grad for p in c64.parameters()]
    res = {}
    xr = torch.nn.functional.pad(xT.t(), (0, 2)).contiguous()   # the kernel's sample-major rows
    for name, fwd in (("fused", lambda: A.critic_grouped(critic, xr)),
                      ("torch", lambda: A.mlp_forward(critic.net, xT.t()).reshape(-1))):
        critic.zero_grad(set_to_none=True)
        v = fwd()
        (v * w).sum().backward()
        res[name] = (float((v.double() - v64).abs().max() / v64.abs().max()),
                     [float((p.grad.double() - g).norm() / g.norm()) for p, g in zip(critic.parameters(), g64)])
    ef, et = res["fused"], res["torch"]
    assert ef[0] <= 3 * et[0] + 1e-7, (ef[0], et[0])
    for a, b in zip(ef[1], et[1]):
        assert a <= max(3 * b, 3e-3), (ef[1], et[1])


def test_shard_keys_kernel_equals_torch(M):
    """fjsp_a2c_shard_keys (the shard learner's combiner keys) equals the torch formula of
    shard_learner.combine's CPU path bit for bit, and flags a non-binary mask byte."""
    A = M["A"]
    SL = __import__("importlib").import_module("multi-agent-rl-for-fjsp_amd.shard_learner")
    import ctypes
    T, n = 5, 1000
    g = torch.Generator().manual_seed(9)
    masks = (torch.rand(T, 29, n, generator=g) < 0.5).to(torch.int8)
    actions = torch.randint(0, 8, (T, 8, n), generator=g, dtype=torch.uint8)
    keys = torch.randint(-2 ** 62, 2 ** 62, (9, T * n), generator=g, dtype=torch.int64)
    info = SL.shard_info_words(masks, actions)
    want = A._fmix64(keys[:8] ^ A._fmix64(info.to(torch.int64) * SL._MIX + 1))
    for bad_byte in (False, True):
        m = masks.clone()
        if bad_byte:
            m[3, 11, 777] = 2
        dm, da, dk = m.cuda(), actions.cuda(), keys.cuda()
        tk = torch.empty(9, T * n, dtype=torch.int64, device="cuda")
        inf = torch.empty(8, T * n, dtype=torch.int32, device="cuda")
        nb = torch.zeros(-(-T * n // 256), dtype=torch.int32, device="cuda")
        V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        A.nat.check(A.nat.lib().fjsp_a2c_shard_keys(V(dk), V(dm), V(da), T, n, V(tk), V(inf), V(nb), None))
        torch.cuda.synchronize()
        assert bool(nb.any()) == bad_byte
        if not bad_byte:
            assert torch.equal(inf.cpu(), info)
            assert torch.equal(tk[:8].cpu(), want)


@pytest.mark.parametrize("k", [3, 8])
def test_record_head_kernel_matches_torch(M, k):
    """fjsp_a2c_record_head (the shard learner's per-record actor loss head) against the same loss
    written in torch ops and differentiated by autograd (shard_learner.owner_losses' CPU path):
    loss and the gradient with respect to the per-input probabilities within f32 rounding, for a
    3-action station and the 8-action AGV, random masks and records of many samples."""
    A = M["A"]
    SL = __import__("importlib").import_module("multi-agent-rl-for-fjsp_amd.shard_learner")
    torch.manual_seed(5)
    U, R = 3000, 50000
    logits = torch.randn(8, U, device="cuda")
    logits[k:] = float("-inf")
    keys = torch.randint(0, U, (R,), device="cuda")
    g = A.RowGroups((keys * 7919 + 11)[None])
    um = g.first.shape[1]
    # the group of input u gets the probabilities of keys[first]: build per-group probabilities
    pu = torch.softmax(logits[:, keys.index_select(0, g.first[0])], dim=0).contiguous().requires_grad_(True)
    bits = torch.randint(0, 1 << k, (R,), device="cuda", dtype=torch.int32)
    act = torch.randint(0, k, (R,), device="cuda", dtype=torch.int32)
    bits |= 1 << act                                  # the action taken is valid (as in a rollout)
    info = (bits | (act << 8)).contiguous()
    wsum = torch.randn(R, device="cuda", dtype=torch.float64) * 5
    cnt = torch.randint(1, 40, (R,), device="cuda", dtype=torch.int32)
    count, coef = 123456.0, 0.01
    got = SL._RecordHead.apply(pu, g, info, wsum, cnt, k, count, coef)
    got.backward()
    g_got = pu.grad.clone()
    pu.grad = None
    p = g.gather(pu[None])
    j = torch.arange(8, device="cuda", dtype=torch.int32)
    m = (((info[None, :] >> j[:, None]) & 1) * (j[:, None] < k)).to(torch.float32)[None]
    ent = A.entropy_of(p)[0]
    logp = A.categorical_log_prob(A.masked_probs(p, m), ((info >> 8) & 0xFF).long()[None])[0]
    want = -(wsum.float() * logp).sum() / count - coef * (cnt.float() * ent).sum() / count
    want.backward()
    ok = torch.isfinite(pu.grad)
    assert abs(float(got) - float(want)) <= 1e-5 * abs(float(want)), (float(got), float(want))
    d = (g_got - pu.grad)[:k][ok[:k]]
    assert float(d.abs().max()) <= 1e-4 * float(pu.grad[:k][ok[:k]].abs().max()), float(d.abs().max())


def test_pack_mfma_kernel_equals_torch(M):
    """fjsp_a2c_pack_mfma (the weights' split-bf16 operand packing, one launch per matrix) equals
    the torch formulation bit for bit: stacked actor layers, the critic's layers, and the
    transposed views the backward packs."""
    A = M["A"]
    g = torch.Generator(device="cuda").manual_seed(2)
    cases = [torch.randn(8, 256, 16, device="cuda", generator=g), torch.randn(8, 256, 256, device="cuda", generator=g),
             torch.randn(256, 48, device="cuda", generator=g) * 1e-3, torch.randn(128, 256, device="cuda", generator=g)]
    cases += [torch.randn(128, 256, device="cuda", generator=g).t(), torch.randn(256, 256, device="cuda", generator=g).t()]
    for W in cases:
        got = A.pack_mfma(W)
        want = A.pack_mfma_torch(W)
        assert got.shape == want.shape
        assert torch.equal(got.view(torch.int32), want.view(torch.int32)), tuple(W.shape)


def test_slab_stats_kernel_matches_torch(M):
    """fjsp_a2c_slab_stats: per-sample sums over the agents of the f32-rounded returns and their
    squares, per-agent sums of the f32-rounded advantages and their squares, against torch f64
    sums of the same values (1e-12 relative: only the f64 summation order differs); partial tiles."""
    A = M["A"]
    g = torch.Generator(device="cuda").manual_seed(6)
    T, N = 37, 1000
    ret = torch.randn(T, 8, N, device="cuda", dtype=torch.float64, generator=g) * 30
    adv = torch.randn(T, 8, N, device="cuda", dtype=torch.float64, generator=g) * 3
    rs, sums = A.slab_stats(ret, adv)
    r32 = ret.float().double()
    assert torch.allclose(rs[0], r32.sum(1).reshape(-1), rtol=1e-12, atol=1e-9)
    assert torch.allclose(rs[1], (r32 * r32).sum(1).reshape(-1), rtol=1e-12, atol=1e-9)
    a32 = adv.float().double()
    want = torch.stack([a32.sum(dim=(0, 2)), (a32 * a32).sum(dim=(0, 2))], dim=1)
    assert torch.allclose(sums, want, rtol=1e-12, atol=1e-9)


def test_critic_onepass_matches_float64(M):
    """The one-pass critic (a2c_vec._CriticOnePass: fjsp_a2c_critic_fused's forward, value
    gradient from the per-state loss coefficients, value-head and hidden-layer backward in one
    kernel, then the split-K weight gradients) against a float64 evaluation of the same loss,
    sum_u a_u/2 V_u^2 + b_u V_u + c_u, beside the three-kernel path (critic_grouped + autograd of
    the same loss): loss within 1e-6 relative, every gradient within max(3x the three-kernel
    path's error, 3e-3) relative (ReLU units within rounding of 0 flip in either f32 path, see
    test_fused_critic_forward_backward_matches_torch); a padding state (0 coefficients)
    contributes nothing."""
    import copy
    A = M["A"]
    torch.manual_seed(4)
    _, critic = A.init_networks(seed=2, device="cuda")
    U = 70001
    xT = (torch.rand(38, U, device="cuda") * torch.randint(0, 30, (38, 1), device="cuda")).float()
    nu = torch.randint(1, 6, (U,), device="cuda").double()
    sr = torch.randn(U, device="cuda", dtype=torch.float64) * nu * 8 * 3
    sr2 = sr * sr / (8 * nu) + torch.rand(U, device="cuda", dtype=torch.float64) * 50
    count = float(nu.sum())
    coef = A.critic_coef_sums(nu, sr, sr2, count)
    coef[-1] = 0.0                                   # a padding state: no samples
    c64 = copy.deepcopy(critic).double()
    v64 = c64.net(xT.double().t()).reshape(-1)
    l64 = (0.5 * coef[:, 0] * v64 * v64 + coef[:, 1] * v64 + coef[:, 2]).sum()
    l64.backward()
    g64 = [p.grad for p in c64.parameters()]
    xr = torch.nn.functional.pad(xT.t(), (0, 2)).contiguous()
    res = {}
    for name, fwd in (("onepass", lambda: A.critic_onepass(critic, xr, coef)),
                      ("three_kernel", lambda: (lambda v: (0.5 * coef[:, 0] * v * v + coef[:, 1] * v + coef[:, 2]).sum())(
                          A.critic_grouped(critic, xr).double()))):
        critic.zero_grad(set_to_none=True)
        loss = fwd()
        loss.backward()
        res[name] = (float(loss), [p.grad.detach().clone() for p in critic.parameters()])
    lo, go = res["onepass"]
    lt, gt = res["three_kernel"]
    assert abs(lo - float(l64)) <= 1e-6 * abs(float(l64)), (lo, float(l64))
    for p_o, p_t, g in zip(go, gt, g64):
        eo = float((p_o.double() - g).norm() / g.norm())
        et = float((p_t.double() - g).norm() / g.norm())
        assert eo <= max(3 * et, 3e-3), (eo, et)


@pytest.mark.parametrize("m,nx,nout,U", [(256, 256, 256, 70001), (128, 256, 256, 33), (256, 40, 38, 70001),
                                         (256, 40, 38, 5), (256, 256, 256, 540017), (128, 256, 256, 540017)])
def test_wgrad_kernel_matches_float64(M, m, nx, nout, U):
    """fjsp_a2c_wgrad (a2c_vec.critic_wgrad: the critic's weight gradients g^T x over the distinct
    states on the matrix cores, split-bf16 products, r06) against float64 for the three layer
    shapes (layer 1 reads the 40-word rows and keeps 38 columns), ragged sample counts (not a
    multiple of the 32-sample stage, fewer stages than workgroups) and a full update's state count:
    relative Frobenius error within max(3x the split-K f32 GEMM's, 2e-6), and bit-identical on a
    second call (the partials are added in a fixed order)."""
    A = M["A"]
    torch.manual_seed(5)
    g = torch.randn(U, m, device="cuda") * (torch.rand(U, m, device="cuda") > 0.5)
    if nx == 40:
        x = torch.nn.functional.pad(torch.rand(U, 38, device="cuda") * 30, (0, 2)).contiguous()
    else:
        x = torch.relu(torch.randn(U, nx, device="cuda"))
    ref = g.double().t() @ x[:, :nout].double()
    gw = A.critic_wgrad(g, x, nout)
    assert gw.shape == (m, nout)
    e = float((gw.double() - ref).norm() / ref.norm())
    et = float((A._splitk_wgrad(g, x[:, :nout]).double() - ref).norm() / ref.norm())
    assert e <= max(3 * et, 2e-6), (e, et)
    assert torch.equal(gw, A.critic_wgrad(g, x, nout))
    assert torch.equal(gw, A._critic_wgrad(g, x, nout if nout != nx else None))
    L = A.nat.lib()
    try:   # the 8-wave kernel (library-wide option "wgrad_waves"): the same bits
        assert L.fjsp_set_option(None, b"wgrad_waves", 8) == 0
        assert torch.equal(gw, A.critic_wgrad(g, x, nout))
    finally:
        assert L.fjsp_set_option(None, b"wgrad_waves", 16) == 0
    if U > 100000:   # the chunked path (batches past the kernel's 2 GiB offset range): the same sum
        old = A.WGRAD_MAX_ROWS
        try:
            A.WGRAD_MAX_ROWS = U // 3 + 5
            gc = A.critic_wgrad(g, x, nout)
        finally:
            A.WGRAD_MAX_ROWS = old
        ec = float((gc.double() - ref).norm() / ref.norm())
        assert ec <= max(3 * et, 2e-6), (ec, et)


def test_prefix_at_equals_full_prefix_sum_on_gpu(M):
    """_prefix_at (the run sums' prefix values at the run ends only, the f64 cast inside the scan)
    is bit-identical to the full f64 prefix sum gathered at the same positions, on the GPU's scan."""
    A = M["A"]
    torch.manual_seed(11)
    for S in (1048576, 70001):
        w = torch.randn(29, S, device="cuda")
        idx = torch.sort(torch.randint(0, S, (29, 4000), device="cuda"), -1).values
        assert torch.equal(torch.gather(A._prefix_sum(w.double()), -1, idx), A._prefix_at(w, idx))


@pytest.mark.parametrize("lowcard", [(), (2, 3, 4, 5, 6, 7), (0, 1, 4, 5, 6), (4,), tuple(range(9))])
def test_row_groups_kernels_equal_stable_sort(M, lowcard):
    """RowGroups on the GPU (fjsp_a2c_group_sort / _runs) equals the grouping by a stable sort of
    each row's 59 key bits computed here in numpy: group counts, the sorted order (equal keys in
    sample order), each sample's group and representative, each group's first sample and run end
    (padding groups: end S, first = the row's last sorted sample).  lowcard: rows grouped by the
    counting sort (<= 64 distinct keys; rows 2, 3, 7 and 8 hold more, so those requests fall back
    to the radix sort for the whole grouping)."""
    import numpy as np
    A = M["A"]
    R, S = 9, 50001
    g = torch.Generator().manual_seed(7)
    card = [3, 28, 1225, 40000, 1, 7, 2, 50001, 600]
    base = torch.stack([torch.randint(0, c, (S,), generator=g) for c in card])
    keys = base * -7046029254386353131 + torch.arange(R)[:, None] * 977   # int64 wrap: keys over all 64 bits
    G = A.RowGroups(keys.cuda(), lowcard)
    k = keys.numpy()
    rows = np.arange(R, dtype=np.int64)[:, None]
    flat = (k & ((1 << 59) - 1)) | (rows << 59)
    order = np.argsort(flat.reshape(-1), kind="stable")
    sk = flat.reshape(-1)[order].reshape(R, S)
    perm = order.reshape(R, S) - rows * S
    new = np.ones((R, S), dtype=bool)
    new[:, 1:] = sk[:, 1:] != sk[:, :-1]
    seg = np.cumsum(new, axis=1) - 1
    U = (seg[:, -1] + 1).tolist()
    assert G.U == U
    umax = G.first.shape[1]
    assert umax == A.bucket(max(U))
    starts = np.full((R, umax), S, dtype=np.int64)
    for r in range(R):
        j = np.nonzero(new[r])[0]
        starts[r, seg[r, j]] = j
    first = perm[rows, np.minimum(starts, S - 1)]
    ends = np.concatenate([starts[:, 1:], np.full((R, 1), S)], axis=1)
    inv = np.empty((R, S), dtype=np.int64)
    inv[rows, perm] = seg
    rep = first[rows, inv]
    for name, want in (("perm", perm), ("inv", inv), ("rep", rep), ("first", first), ("ends", ends)):
        assert np.array_equal(getattr(G, name).cpu().numpy(), want), name


@pytest.mark.parametrize("S", [1, 63, 1024, 1025, 1048576])
def test_row_groups_counting_sort_equals_radix(M, S):
    """The station rows' counting sort (lowcard) at the A2C batch's size: every output of the
    grouping equal to the radix sort's, with rows of 1, 2, 30 and 64 distinct keys (the counting
    path's limit), a skewed row and partial 1 024-sample chunks."""
    A = M["A"]
    g = torch.Generator().manual_seed(11)
    cols = [torch.zeros(S, dtype=torch.int64), torch.randint(0, 2, (S,), generator=g),
            torch.randint(0, 30, (S,), generator=g), torch.randint(0, 64, (S,), generator=g),
            (torch.rand(S, generator=g) ** 8 * 40).long(), torch.randint(0, 5000, (S,), generator=g)]
    keys = (torch.stack(cols) * -7046029254386353131 + 12345).cuda()
    a = A.RowGroups(keys, (0, 1, 2, 3, 4))
    b = A.RowGroups(keys)
    assert a.U == b.U
    for name in ("perm", "inv", "rep", "first", "ends", "gsorted"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


@pytest.mark.parametrize("S", [1, 1023, 50001, 300000, 1300000])
def test_run_sums_kernel_equals_float64_group_sums(M, S):
    """fjsp_a2c_run_sums (the per-group gradient sums of the grouped update, one pass over the
    sorted runs) against float64 group sums of the same f32 products: groups of one sample,
    groups spanning many 1 024-position chunks, a row that is one group, scaled rows; within one
    f32 rounding of the f64 sum (+ f64 summation error).  The _GatherRuns backward (_run_sums)
    takes the same kernel.  S = 1 300 000 has 1 270 chunks per row, so k_run_carry's second tile
    of 1 024 chunks runs (the gather learner's 8.4 M samples have 8 192): the one-group row and
    the 3-group row's runs carry their sums across the tile boundary."""
    A = M["A"]
    R = 5
    g = torch.Generator().manual_seed(S)
    card = [1, 3, 977, max(1, S // 2), S]
    base = torch.stack([torch.randint(0, c, (S,), generator=g) for c in card])
    G = A.RowGroups((base * -7046029254386353131 + torch.arange(R)[:, None]).cuda())
    assert G.gsorted is not None
    J = 9
    rowmap = torch.tensor([0, 1, 2, 3, 4, 4, 3, 1, 2], dtype=torch.int32)
    vals = torch.randn(J, S, generator=g) * torch.logspace(-3, 3, J)[:, None]
    scale = torch.rand(J, generator=g) + 0.5
    got = A.run_sums(vals.cuda(), rowmap.cuda(), scale.cuda(), G).cpu().double()
    umax = G.first.shape[1]
    assert got.shape == (J, umax)
    inv = G.inv.cpu()
    x = (vals * scale[:, None]).double()
    want = torch.zeros(J, umax, dtype=torch.float64)
    mag = torch.zeros(J, umax, dtype=torch.float64)
    for j in range(J):
        want[j].index_add_(0, inv[int(rowmap[j])], x[j])
        mag[j].index_add_(0, inv[int(rowmap[j])], x[j].abs())
    tol = torch.finfo(torch.float32).eps * want.abs() + 1e-12 * mag + 1e-300
    assert bool(((got - want).abs() <= tol).all()), float(((got - want).abs() / (want.abs() + 1e-30)).max())
    gy = vals[:3].reshape(1, 3, S).expand(R, 3, S).contiguous().cuda()
    a = A._run_sums(G, gy).cpu().double()
    for r in range(R):
        for c in range(3):
            w = torch.zeros(umax, dtype=torch.float64).index_add_(0, inv[r], vals[c].double())
            m = torch.zeros(umax, dtype=torch.float64).index_add_(0, inv[r], vals[c].double().abs())
            assert bool(((a[r, c] - w).abs() <= torch.finfo(torch.float32).eps * w.abs() + 1e-12 * m + 1e-300).all())
