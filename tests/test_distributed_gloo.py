"""Multi-process (world_size 2, gloo on CPU) coverage of the N>1 path:
sharded A2C update == single-learner update over the concatenated batch (one flat gradient
all_reduce + global advantage statistics), experience all_gather, max-over-ranks timing and
the env-shard id ranges bench.py uses."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
D = importlib.import_module("multi-agent-rl-for-fjsp_amd.distributed")

from tests.parity_util import assert_grads_close  # noqa: E402

T, N = 16, 24           # batch of T steps x N envs, split N/2 per rank


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(seed=0):
    g = torch.Generator().manual_seed(seed)
    feats = torch.randint(0, 6, (T, 38, N), generator=g).float()
    feats[:, 21::3] = torch.rand(T, 6, N, generator=g)
    masks = (torch.rand(T, 29, N, generator=g) < 0.6).to(torch.int8)
    for off in A.MASK_OFFS:
        masks[:, off] = 1
    acts = torch.zeros(T, 8, N, dtype=torch.uint8)
    for a in range(8):   # a valid action per agent
        m = masks[:, A.MASK_OFFS[a]:A.MASK_OFFS[a] + A.N_ACTIONS[a]].float()
        acts[:, a] = torch.multinomial(m.permute(0, 2, 1).reshape(-1, A.N_ACTIONS[a]), 1, generator=g).view(T, N).to(torch.uint8)
    ret = torch.randn(T, 8, N, generator=g, dtype=torch.float64) * 20
    adv = torch.randn(T, 8, N, generator=g, dtype=torch.float64) * 3
    return feats, masks, acts, ret, adv


def _update(feats, masks, acts, ret, adv, group=None):
    actors, critic = A.init_networks(seed=11)
    oa = torch.optim.Adam(actors.parameters(), lr=3e-4)
    oc = torch.optim.Adam(critic.parameters(), lr=1e-3)
    grads = []
    al, cl = A.update_step(actors, critic, oa, oc, feats, masks, acts, ret, adv, A.gather_index("cpu"),
                           A.mask_index("cpu"), 0.01, 0.5, group, grad_probe=grads.append)
    params = torch.cat([p.detach().reshape(-1) for p in list(actors.parameters()) + list(critic.parameters())])
    return al, cl, params, grads[0]


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    feats, masks, acts, ret, adv = _batch()
    base, n = D.shard_range(N // world, rank)
    sl = slice(base, base + n)
    al, cl, params, grads = _update(feats[..., sl].contiguous(), masks[..., sl].contiguous(),
                                    acts[..., sl].contiguous(), ret[..., sl].contiguous(), adv[..., sl].contiguous(),
                                    group=dist.group.WORLD)
    slab = torch.full((3, 5), float(rank))
    gathered = D.gather_transitions(slab)
    tmax = D.allreduce_max(torch.tensor([1.5 + rank]))
    torch.save({"al": al, "cl": cl, "params": params, "grads": grads, "gathered": gathered, "tmax": tmax},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def two_rank_results(tmp_path_factory):
    out = tmp_path_factory.mktemp("gloo")
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    return [torch.load(os.path.join(out, f"rank{r}.pt"), weights_only=True) for r in range(2)]


def test_sharded_update_equals_single_learner(two_rank_results):
    r0, r1 = two_rank_results
    al, cl, params, grads = _update(*_batch())
    for r in (r0, r1):
        assert np.allclose(r["al"], al, rtol=1e-4, atol=1e-6)
        assert r["cl"] == pytest.approx(cl, rel=1e-5)
        # the all-reduced gradients (before clipping / Adam) are the single learner's
        assert_grads_close(r["grads"], grads)
    # replicated parameters stay identical across ranks
    assert torch.equal(r0["params"], r1["params"])
    assert torch.equal(r0["grads"], r1["grads"])


def test_gather_and_max(two_rank_results):
    for r in two_rank_results:
        g = r["gathered"]
        assert g.shape == (2, 3, 5) and bool((g[0] == 0).all()) and bool((g[1] == 1).all())
        assert float(r["tmax"][0]) == 2.5


def test_shard_ranges_cover_global_ids():
    ids = []
    for rank in range(8):
        base, n = D.shard_range(4096, rank)
        ids.extend(range(base, base + n))
    assert ids == list(range(8 * 4096))


# ---------------------------------------------------------------- experience gather (exchange="gather")
class _CpuEnv:
    """Stand-in for FJSPVecEnv in the CPU test: the learner only needs the device, the shard
    size and its global id base here (the transitions are given)."""

    def __init__(self, n, base):
        self.device = torch.device("cpu")
        self.num_envs = n
        self.env_id_base = base

    def faults(self, clear=False):
        return 0


def _gae_cpu(rewards, values, done, gamma, lamb, use_gae=True):
    """transition_memory.py:83-105 in torch fp64 (test stand-in for the GAE kernel)."""
    T, _, n = rewards.shape
    v = values.double()
    ret = torch.zeros_like(rewards)
    adv = torch.zeros_like(rewards)
    r_acc = v[T].expand(8, n).clone()
    g_acc = torch.zeros(8, n, dtype=torch.float64)
    nxt = v[T].expand(8, n).clone()
    for t in range(T - 1, -1, -1):
        end = done[t].bool().expand(8, n)
        r_acc = torch.where(end, torch.zeros_like(r_acc), r_acc)
        g_acc = torch.where(end, torch.zeros_like(g_acc), g_acc)
        nv = torch.where(end, torch.zeros_like(nxt), nxt)
        r_acc = rewards[t] + gamma * r_acc
        delta = (rewards[t] + gamma * nv) - v[t].expand(8, n)
        g_acc = delta + (gamma * lamb) * g_acc
        ret[t], adv[t] = r_acc, g_acc
        nxt = v[t].expand(8, n)
    return ret, adv


def _rollout_batch(seed=0):
    feats, masks, acts, _, _ = _batch(seed)
    g = torch.Generator().manual_seed(seed + 1)
    feats = torch.cat([feats, feats[-1:]], dim=0)                 # [T + 1, 38, N]
    masks = torch.cat([masks, masks[-1:]], dim=0)
    values = torch.randn(T + 1, N, generator=g) * 5
    rewards = torch.randn(T, 8, N, generator=g, dtype=torch.float64)
    term = (torch.rand(T, N, generator=g) < 0.05).to(torch.uint8)
    trunc = torch.zeros(T, N, dtype=torch.uint8)
    return dict(feats=feats, masks=masks, actions=acts, values=values, rewards=rewards, term=term, trunc=trunc)


def _learner(n, base, group, exchange):
    L = A.VecMultiAgentA2C(_CpuEnv(n, base), batch_size=T, seed=11, group=group, use_graph=False,
                           fused_policy=False, exchange=exchange)
    L.gae_fn = _gae_cpu     # CPU stand-in for the GAE kernel (this learner's only GPU call), per instance
    L._alloc()
    return L


def _fill(L, sl):
    for k, v in _rollout_batch().items():
        L._bufs[k].copy_(v[..., sl])


def _gather_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    n = N // world
    L = _learner(n, rank * n, dist.group.WORLD, "gather")
    _fill(L, slice(rank * n, (rank + 1) * n))
    grads = []
    L.grad_probe = grads.append
    al, cl = L.update()
    params = torch.cat([p.detach().reshape(-1) for p in list(L.actors.parameters()) + list(L.critic.parameters())])
    slabs = D.gather_slabs({"a": torch.full((2, 3), rank, dtype=torch.int16),
                            "b": torch.full((4,), 0.5 + rank, dtype=torch.float64)}, dst=0)
    if slabs is not None:     # views of one receive buffer (different dtypes): saved as copies
        slabs = {k: v.clone() for k, v in slabs.items()}
    torch.save({"al": al, "cl": cl, "params": params, "slabs": slabs, "grads": grads},
               os.path.join(out_dir, f"g{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_exchange_equals_single_learner(tmp_path):
    """exchange="gather": the learner rank's update over the gathered batch IS the single
    learner's update (same data, same ops), and the broadcast hands it to every rank."""
    mp.spawn(_gather_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [torch.load(os.path.join(tmp_path, f"g{k}.pt"), weights_only=True) for k in range(2)]
    L = _learner(N, 0, None, "allreduce")
    _fill(L, slice(0, N))
    grads = []
    L.grad_probe = grads.append
    al, cl = L.update()
    params = torch.cat([p.detach().reshape(-1) for p in list(L.actors.parameters()) + list(L.critic.parameters())])
    assert torch.equal(r[0]["params"], r[1]["params"])      # the broadcast replicated the learner's update
    assert len(r[0]["grads"]) == 1 and r[1]["grads"] == []   # only the learner rank computes gradients
    assert_grads_close(r[0]["grads"][0], grads[0])           # same data and ops; the CPU GEMMs' thread
    #                                                          count differs (reduction order only)
    for k in range(2):
        assert np.allclose(r[k]["al"], al, rtol=1e-5, atol=1e-7) and r[k]["cl"] == pytest.approx(cl, rel=1e-5)
    s = r[0]["slabs"]
    assert s["a"].shape == (2, 2, 3) and bool((s["a"][1] == 1).all()) and bool((s["a"][0] == 0).all())
    assert s["b"].dtype == torch.float64 and float(s["b"][1, 0]) == 1.5
    assert r[1]["slabs"] is None


# ---------------------------------------------------------------- learner sharded by network (exchange="shard")
def _shard_worker(rank, world, port, out_dir, collide=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    if collide:   # 4-bit grouping keys: different inputs collide, the combiner's check must catch it
        gk = A.group_keys
        A.group_keys = lambda f3, rows=None: gk(f3, rows) & 0xF
    n = N // world
    L = _learner(n, rank * n, dist.group.WORLD, "shard")
    _fill(L, slice(rank * n, (rank + 1) * n))
    grads = []
    L.grad_probe = grads.append
    al, cl = L.update()
    params = torch.cat([p.detach().reshape(-1) for p in list(L.actors.parameters()) + list(L.critic.parameters())])
    torch.save({"al": al, "cl": cl, "params": params, "grads": grads, "info": L.shard_info},
               os.path.join(out_dir, f"s{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_shard_exchange_equals_single_learner(tmp_path, world):
    """exchange="shard": each rank combines its samples into (input, mask, action) / global-state
    records, one all_to_all routes them to the rank owning the network (actor a on rank a mod
    world, critic states by key), owners back-propagate, one all_reduce sums the gradients: the
    single learner's gradients up to summation order, identical parameters on every rank."""
    assert N % world == 0
    mp.spawn(_shard_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [torch.load(os.path.join(tmp_path, f"s{k}.pt"), weights_only=True) for k in range(world)]
    L = _learner(N, 0, None, "allreduce")
    _fill(L, slice(0, N))
    grads = []
    L.grad_probe = grads.append
    al, cl = L.update()
    params = torch.cat([p.detach().reshape(-1) for p in list(L.actors.parameters()) + list(L.critic.parameters())])
    for k in range(world):
        assert not r[k]["info"]["fallback"]
        assert len(r[k]["grads"]) == 1
        assert_grads_close(r[k]["grads"][0], grads[0])
        assert torch.equal(r[k]["grads"][0], r[0]["grads"][0])   # one all_reduce: the same sums everywhere
        assert torch.equal(r[k]["params"], r[0]["params"])
        assert np.allclose(r[k]["al"], al, rtol=1e-5, atol=1e-7) and r[k]["cl"] == pytest.approx(cl, rel=1e-5)
    assert torch.allclose(r[0]["params"], params, rtol=0, atol=1e-6)
    # every sample went into exactly one actor record per agent and one critic record
    assert sum(x["info"]["samples"] for x in r) == T * N
    assert sum(x["info"]["critic_records_received"] for x in r) == sum(x["info"]["critic_records_sent"] for x in r)


def test_shard_exchange_hash_collision_falls_back(tmp_path):
    """A hash collision in the combiner's grouping (forced: 4-bit keys) is caught by the bitwise
    check against the representatives, flagged through the gradient all_reduce, and every rank
    redoes the batch with the all-reduce exchange (whose own grouping check then takes the dense
    update): the single learner's gradients, identical parameters on every rank."""
    world = 2
    mp.spawn(_shard_worker, args=(world, _free_port(), str(tmp_path), True), nprocs=world, join=True)
    r = [torch.load(os.path.join(tmp_path, f"s{k}.pt"), weights_only=True) for k in range(world)]
    L = _learner(N, 0, None, "allreduce")
    _fill(L, slice(0, N))
    grads = []
    L.grad_probe = grads.append
    L.update()
    for k in range(world):
        assert r[k]["info"]["fallback"]
        assert_grads_close(r[k]["grads"][0], grads[0])
        assert torch.equal(r[k]["params"], r[0]["params"])
