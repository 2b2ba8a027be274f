"""RCCL (torch.distributed "nccl" on ROCm) executed on one GPU: a single-rank nccl group with
distributed.FORCE_ACTIVE set, so that every collective branch the multi-GPU job takes — the
device-tensor paths of gather_slabs, broadcast_flat, allreduce_grads, adv_stats_slab,
max_over_ranks and the shard exchange's all_to_all / all_reduce — runs through RCCL on device
tensors (the CPU suite drives them with gloo on host tensors only).  A world of one leaves every
result equal to its input, and each learner exchange equal to the single learner (a2c.py:324-336,
647-731)."""
import importlib
import os
import socket

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from tests.parity_util import assert_grads_close  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def R():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import torch.distributed as dist
    D = importlib.import_module("multi-agent-rl-for-fjsp_amd.distributed")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    assert dist.get_backend() == "nccl"
    D.FORCE_ACTIVE = True
    try:
        yield D
    finally:
        D.FORCE_ACTIVE = False
        dist.destroy_process_group()


def test_rccl_collective_helpers_on_device_tensors(R):
    D = R
    dev = torch.device("cuda:0")
    assert D.active(None) and D._backend(None) == "nccl"
    g = torch.Generator(device=dev).manual_seed(3)
    slabs = {"f": torch.rand(5, 7, 64, device=dev, generator=g),
             "m": (torch.rand(5, 3, 64, device=dev, generator=g) < 0.5).to(torch.int8),
             "a": torch.randint(0, 8, (5, 9), device=dev, generator=g, dtype=torch.uint8),
             "r": torch.randn(5, 8, 64, device=dev, generator=g, dtype=torch.float64)}
    out = D.gather_slabs(slabs, dst=0)
    assert list(out) == list(slabs)
    base = out["r"].untyped_storage().data_ptr()
    for k, v in slabs.items():
        assert out[k].shape == (1,) + v.shape and out[k].dtype == v.dtype and out[k].is_cuda
        assert torch.equal(out[k][0], v), k
        assert out[k].untyped_storage().data_ptr() == base      # views of one receive buffer, no copies
    ts = [torch.randn(4, 4, device=dev, generator=g), torch.randn(3, device=dev, generator=g)]
    before = [t.clone() for t in ts]
    D.broadcast_flat(ts, src=0)
    assert all(torch.equal(a, b) for a, b in zip(ts, before))
    lin = torch.nn.Linear(6, 3).to(dev)
    lin(torch.randn(9, 6, device=dev, generator=g)).sum().backward()
    gb = [p.grad.clone() for p in lin.parameters()]
    D.allreduce_grads(list(lin.parameters()))
    assert all(torch.equal(p.grad, q) for p, q in zip(lin.parameters(), gb))
    adv = torch.randn(16, 8, 512, device=dev, generator=g, dtype=torch.float64)
    n, mean, std = D.adv_stats_slab(adv)
    x = adv.float().permute(1, 0, 2).reshape(8, -1)
    assert n == 16 * 512
    assert torch.allclose(mean, x.mean(1), rtol=1e-6, atol=1e-7) and torch.allclose(std, x.std(1), rtol=1e-6)
    assert D.max_over_ranks(5, None, dev) == 5
    t = D.gather_transitions(torch.arange(6.0, device=dev).view(2, 3))
    assert t.shape == (1, 2, 3) and torch.equal(t[0], torch.arange(6.0, device=dev).view(2, 3))


def _learner(exchange, n=256, T=64):
    A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
    V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
    import torch.distributed as dist
    L = A.VecMultiAgentA2C(V.FJSPVecEnv(n), batch_size=T, seed=7, group=dist.group.WORLD, exchange=exchange)
    L.reset(seeds=torch.arange(n), num_orders=25)
    L.collect()
    return L


SHARD_STAGES = ("gae", "adv_stats", "combine", "exchange", "own", "all_reduce", "clip_adam")


@pytest.mark.timeout(300)
def test_rccl_learner_exchanges_equal_single_learner(R):
    """The three exchanges through RCCL with one rank: "gather" is the single learner's update on
    the same bytes (bit-equal gradients), "allreduce" and "shard" equal it up to summation order."""
    D = R
    res = {}
    for ex in ("local", "gather", "allreduce", "shard"):
        L = _learner("allreduce" if ex == "local" else ex)
        grads = []
        L.grad_probe = grads.append
        if ex == "local":
            D.FORCE_ACTIVE = False      # the plain single learner: no collective at all
            try:
                L.update()
            finally:
                D.FORCE_ACTIVE = True
        else:
            if ex == "shard":
                L.exchange_timing = {}   # the bench's synchronised stage timers
            L.update()
            if ex == "shard":
                assert set(L.exchange_timing) == {"learn"} | {"shard_" + k for k in SHARD_STAGES}, L.exchange_timing
                assert all(v >= 0 for v in L.exchange_timing.values())
                L.exchange_timing = None
        p = torch.cat([q.detach().reshape(-1) for q in list(L.actors.parameters()) + list(L.critic.parameters())])
        res[ex] = (grads[0], p, L.critic_loss_history[-1], [h[-1] for h in L.actor_loss_history.values()],
                   dict(L.shard_info), L._bufs["rewards"].clone())
        del L
    ref = res["local"]
    for ex in ("gather", "allreduce", "shard"):
        g, p, cl, al, info, rw = res[ex]
        assert torch.equal(rw, ref[5]), ex                 # the same batch (same seeds and draws)
        if ex == "gather":
            assert torch.equal(g, ref[0])
        else:
            assert_grads_close(g, ref[0])
        assert cl == pytest.approx(ref[2], rel=1e-5), ex
        assert all(abs(a - b) <= 1e-4 * abs(b) + 1e-6 for a, b in zip(al, ref[3])), ex
    info = res["shard"][4]
    assert not info["fallback"] and info["bytes_sent_to_other_ranks"] == 0
    assert info["samples"] == 64 * 256
    assert info["critic_records_received"] == info["critic_records_sent"] > 0
