"""BASELINE config 5 on one GPU: env shards keyed by global id.

* Two handles with env_id_base 0 and N produce the bytes of one 2N handle, and the shard at
  base N the bytes of the oracle at gid0 = N (FJSPSimulation seeded np.random.seed(gid), actions
  keyed by gid), across truncation / all-orders-done auto-resets, through the fused kernels
  (k_step_ag, k_step_pipe) and the one-launch-per-step kernel.
* An A2C learner on the shard [n, 2n) collects exactly the second half of a 2n-env learner's
  first batch (same seed: MT streams and policy draws keyed by global id).
* Two ranks (gloo, both on cuda:0, launched by torch.distributed.run as fresh processes) train
  with either exchange (gradient all_reduce / experience gather into the learner) and match one
  learner over all 2n envs (reference: a2c.py:324-336, memory -> finish_trajectory -> _update).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import parity_util as P  # noqa: E402

LEAN = ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "status")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from tests import gpu_util
    return gpu_util


def _rollout(G, env, steps, policy, seed=77):
    return G.to_np(env.rollout(steps, action_seed=seed, policy=policy))


@pytest.mark.parametrize("policy,num_orders", [("random", 30), ("masked", 3), ("heuristic", 2)])
def test_shards_equal_one_handle_and_oracle(G, policy, num_orders):
    N, steps = 96, 420                        # 96: a partial 64-env workgroup per shard
    big = G.vec_env.FJSPVecEnv(2 * N)
    shards = [G.vec_env.FJSPVecEnv(N, env_id_base=r * N) for r in range(2)]
    for e in [big] + shards:
        e.reset(num_orders=num_orders)        # seed=None: default streams np.random.seed(gid)
    rb = _rollout(G, big, steps, policy)
    rs = [_rollout(G, s, steps, policy) for s in shards]
    for k in LEAN:
        cat = np.concatenate([r[k] for r in rs], axis=1)
        assert np.array_equal(rb[k], cat), (policy, k)
    ends = int((rb["term"] | rb["trunc"]).sum())
    assert ends >= 2 * N                      # every env crossed at least one auto-reset
    # the shard at base N == the oracle's envs N..2N-1 (its own gid-keyed seeds and actions)
    opol = {"random": 0, "masked": 1, "heuristic": 3}[policy]
    rec, _, _ = O.rollout(N, steps, gid0=N, num_orders=num_orders, action_seed=77, policy=opol)
    for k in LEAN:
        if k == "status":
            continue
        ref = rec[k] if rec[k].ndim == 3 else rec[k]
        assert np.array_equal(rs[1][k], ref.reshape(rs[1][k].shape)), (policy, k)


def test_shards_per_step_kernel(G):
    """fjsp_step (actions from HBM, one launch per step) on the shards == on one handle."""
    N, steps = 80, 230
    big = G.vec_env.FJSPVecEnv(2 * N)
    shards = [G.vec_env.FJSPVecEnv(N, env_id_base=r * N) for r in range(2)]
    for e in [big] + shards:
        e.reset(num_orders=30)
    g = torch.Generator(device="cuda").manual_seed(3)
    nact = torch.tensor([3, 8, 3, 3, 3, 3, 3, 3], device="cuda").view(8, 1)
    for t in range(steps):
        a = (torch.randint(0, 1 << 20, (8, 2 * N), device="cuda", generator=g) % nact).to(torch.uint8)
        ob = G.to_np(big.step(a))
        os_ = [G.to_np(s.step(a[:, r * N:(r + 1) * N].contiguous())) for r, s in enumerate(shards)]
        for k in LEAN + ("next_i32", "next_masks"):
            assert np.array_equal(ob[k], np.concatenate([o[k] for o in os_], axis=1)), (t, k)


def test_a2c_shard_collect_matches_big(G):
    A = __import__("importlib").import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
    n, T = 64, 24
    big = A.VecMultiAgentA2C(G.vec_env.FJSPVecEnv(2 * n), batch_size=T, seed=9)
    shard = A.VecMultiAgentA2C(G.vec_env.FJSPVecEnv(n, env_id_base=n), batch_size=T, seed=9)
    for L in (big, shard):
        L.reset(num_orders=25)
        L.collect()
    torch.cuda.synchronize()
    for k in ("feats", "masks", "actions", "values", "rewards", "term", "trunc"):
        assert torch.equal(big._bufs[k][..., n:], shard._bufs[k]), k


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _single_learner(n_total, T, batches):
    """One learner over all n_total envs (seed 5, as every rank): its first batch's buffers, the
    gradients of its first update before clipping / Adam, and the learner."""
    A = __import__("importlib").import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
    V = __import__("importlib").import_module("multi-agent-rl-for-fjsp_amd.vec_env")
    L = A.VecMultiAgentA2C(V.FJSPVecEnv(n_total), batch_size=T, seed=5)
    L.reset(num_orders=25)
    first, grads = None, []
    for i in range(batches):
        L.collect()
        if i == 0:
            first = {k: L._bufs[k].cpu().clone() for k in ("feats", "masks", "actions", "values", "rewards", "term",
                                                             "trunc")}
            L.grad_probe = lambda g: grads.append(g.cpu())
        L.update()
        L.grad_probe = None
        L.roll_over()
    return first, grads[0], L


def run_ranks(world, n, T, batches, exchange, out, digest=False, timeout=240):
    """world ranks (gloo, every rank on cuda:0) as fresh processes under torch.distributed.run."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "tests", "dist_a2c_worker.py"),
           "--shard-envs", str(n), "--shard-batch", str(T), "--shard-batches", str(batches), "--shard-exchange", exchange,
           "--shard-out", str(out)] + (["--shard-digest"] if digest else [])
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [torch.load(out / f"rank{k}.pt", weights_only=True) for k in range(world)]


@pytest.mark.parametrize("exchange", ["allreduce", "gather", "shard"])
def test_two_rank_a2c_equals_single_learner(G, tmp_path, exchange):
    n, T = 64, 32
    ranks = run_ranks(2, n, T, 2, exchange, tmp_path)
    first, grads, L = _single_learner(2 * n, T, 2)
    # batch 1: the shards' rollouts are the halves of the single learner's (bit for bit)
    for k, rk in enumerate(ranks):
        for f, v in rk["first"].items():
            assert torch.equal(first[f][..., k * n:(k + 1) * n], v), (exchange, k, f)
    # the reduced gradients of the first update (before clipping and Adam) are the single
    # learner's: per tensor ||g - g_ref|| <= 1e-5 ||g_ref|| (all-reduce: every rank; gather:
    # the learner rank, the others compute none)
    P.assert_grads_close(ranks[0]["grads1"], grads)
    if exchange in ("allreduce", "shard"):
        assert torch.equal(ranks[0]["grads1"], ranks[1]["grads1"])
    else:
        assert ranks[1]["grads1"] is None
    # the replicated parameters agree across ranks (both batches)
    assert torch.equal(ranks[0]["params"], ranks[1]["params"])
    assert torch.equal(ranks[0]["params1"], ranks[1]["params1"])
    assert bool(torch.isfinite(ranks[0]["params"]).all())
    assert ranks[0]["critic"][0] == pytest.approx(L.critic_loss_history[0], rel=1e-5)
    for a in range(8):
        assert ranks[0]["actor"][a][0] == pytest.approx(L.actor_loss_history[list(L.actor_loss_history)[a]][0],
                                                        rel=1e-4, abs=1e-6)
    if exchange == "gather":
        assert ranks[0]["exchange_bytes"] == T * n * 258 + n * 4
