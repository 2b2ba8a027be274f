#!/usr/bin/env python3
"""Config 5's learner sharded by network (exchange="shard", shard_learner.py), every rank's share
timed alone on one GPU, and its gradients against one learner over all the envs.

One 32 768-env learner collects a 256-step batch (after `warm` batches of training, so the state
distribution is a training one).  The batch is cut into `world` env shards of 4 096 (exactly what
the ranks of a config-5 job hold); each shard's combiner runs timed (GAE + statistics + keys +
grouping + records), the all_to_all is emulated in-process (shard_learner.emulate), each owner's
share runs timed (regrouping, its actors and its part of the critic, backward), and the summed
gradients are compared per tensor with the single learner's (grad_probe).  The per-rank learner
share = combine + own (+ the clip / Adam step, timed once).  Prints one JSON line."""
import importlib
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
D = importlib.import_module("multi-agent-rl-for-fjsp_amd.distributed")
SL = importlib.import_module("multi-agent-rl-for-fjsp_amd.shard_learner")
from tests.parity_util import grad_errors  # noqa: E402


def sync_ms(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    return out, (time.perf_counter() - t0) * 1e3


def main(world=8, n=4096, T=256, warm=1, reps=3):
    N = world * n
    L = A.VecMultiAgentA2C(V.FJSPVecEnv(N), batch_size=T, seed=5)
    L.reset(num_orders=25)
    for _ in range(warm):
        L.collect()
        L.update()
        L.roll_over()
    L.collect()
    torch.cuda.synchronize()
    b = L._bufs
    shards = []
    for r in range(world):
        sl = slice(r * n, (r + 1) * n)
        shards.append({k: b[k][..., sl].contiguous() for k in ("feats", "masks", "actions", "rewards", "values")}
                      | {"done": (b["term"] | b["trunc"])[..., sl].contiguous()})
    # the global advantage statistics (the all_reduce of adv_stats_slab) from every shard's GAE
    rets = [L.gae_fn(s["rewards"], s["values"], s["done"], L.gamma, L.lamb, L.use_gae) for s in shards]
    count, mean, std = D.adv_stats_slab(torch.cat([a for _, a in rets], dim=2))
    res = {"world": world, "envs_per_rank": n, "batch": T, "warm_batches": warm}
    for rep in range(reps):
        t_comb, t_gae, combs = [], [], []
        for r, s in enumerate(shards):
            (ret, adv), tg = sync_ms(lambda: L.gae_fn(s["rewards"], s["values"], s["done"], L.gamma, L.lamb, L.use_gae))
            c, tc = sync_ms(lambda: SL.combine(s["feats"][:T], s["masks"][:T], s["actions"], ret, adv, mean, std, world))
            t_gae.append(tg)
            t_comb.append(tc)
            combs.append(c)
        recvs = SL.emulate(combs)
        t_own, gsum = [], None
        info = []
        for d in range(world):
            L.optim_actor.zero_grad(set_to_none=True)
            L.optim_critic.zero_grad(set_to_none=True)

            def own():
                al, cl, bad = SL.owner_losses(L.actors, L.critic, recvs[d], d, world, count, L.entropy_coef)
                if al.requires_grad or cl.requires_grad:
                    (al.sum() + cl).backward()
                return al, cl, bad
            (al, cl, bad), to = sync_ms(own)
            t_own.append(to)
            g = A.flat_grads(L.actors, L.critic).double()
            gsum = g if gsum is None else gsum + g
            info.append({"actor_records": int(recvs[d][0].shape[0]), "critic_records": int(recvs[d][1].shape[0]),
                         "bad": float(bad)})
        share = [t_gae[r] + t_comb[r] + t_own[r] for r in range(world)]
        res["rep%d" % rep] = {"gae_ms": t_gae, "combine_ms": t_comb, "own_ms": t_own, "share_ms": share,
                              "max_share_ms": max(share)}
    res["owners"] = info
    prof = os.environ.get("FJSP_PROFILE_SHARE")
    if prof is not None:   # a torch-profiler table of one rank's combine + own (device time per op)
        from torch.profiler import ProfilerActivity, profile
        d = int(prof)
        s = shards[d]
        L.optim_actor.zero_grad(set_to_none=True)
        L.optim_critic.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as pr:
            ret, adv = L.gae_fn(s["rewards"], s["values"], s["done"], L.gamma, L.lamb, L.use_gae)
            SL.combine(s["feats"][:T], s["masks"][:T], s["actions"], ret, adv, mean, std, world)
            torch.cuda.synchronize()
        print("== combine (rank %d)" % d, file=sys.stderr)
        print(pr.key_averages().table(sort_by="self_cuda_time_total", row_limit=30), file=sys.stderr)
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as pr:
            al, cl, bad = SL.owner_losses(L.actors, L.critic, recvs[d], d, world, count, L.entropy_coef)
            (al.sum() + cl).backward()
            torch.cuda.synchronize()
        print("== own (rank %d)" % d, file=sys.stderr)
        print(pr.key_averages().table(sort_by="self_cuda_time_total", row_limit=30), file=sys.stderr)
    res["bytes_sent_to_other_ranks"] = [sum(c.bytes_by_dest()) - c.bytes_by_dest()[r] for r, c in enumerate(combs)]
    res["bytes_by_dest_rank0"] = combs[0].bytes_by_dest()
    res["gather_bytes_per_rank"] = L.exchange_bytes_per_batch() // world if L.exchange == "gather" else T * n * 258 + n * 4
    # the single learner over all N envs on the same batch (grad_probe before clip / Adam)
    grads = []
    L.grad_probe = grads.append
    _, t_single = sync_ms(lambda: L.update())
    errs = grad_errors(gsum.float(), grads[0])
    res["single_learner_update_ms"] = t_single
    res["max_rel_grad_error"] = max(e for _, e in errs)
    res["rel_grad_error_per_tensor"] = [[list(s), e] for s, e in errs]
    # clip + Adam (every rank runs it on the reduced gradients)
    _, t_adam = sync_ms(lambda: (A.clip_per_agent_(L.actors, L.max_grad_norm),
                                 torch.nn.utils.clip_grad_norm_(L.critic.parameters(), L.max_grad_norm),
                                 L.optim_actor.step(), L.optim_critic.step()))
    res["clip_adam_ms"] = t_adam
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:]))
