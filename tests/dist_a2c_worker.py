"""One rank of the 2-rank A2C rehearsal of BASELINE config 5 (run by tests/test_gpu_shards.py
under torch.distributed.run; gloo between the ranks, every rank on cuda:0).

Rank r steps the env shard [r*n, (r+1)*n) (FJSPVecEnv(env_id_base=r*n)) and trains with the
exchange given on the command line; it saves its first batch's rollout buffers, the loss
histories and the final parameters for the parent test to compare with one learner over 2n
envs."""
import argparse
import importlib
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def flat(L):
    return torch.cat([p.detach().reshape(-1).cpu() for p in list(L.actors.parameters()) + list(L.critic.parameters())])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard-envs", type=int, required=True)
    ap.add_argument("--shard-batch", type=int, required=True)
    ap.add_argument("--shard-batches", type=int, default=2)
    ap.add_argument("--shard-exchange", default="allreduce")
    ap.add_argument("--shard-out", required=True)
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
    A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
    env = V.FJSPVecEnv(a.shard_envs, device="cuda:0", env_id_base=rank * a.shard_envs)
    L = A.VecMultiAgentA2C(env, batch_size=a.shard_batch, seed=5, group=dist.group.WORLD, exchange=a.shard_exchange)
    L.reset(num_orders=25)
    first = None
    for i in range(a.shard_batches):
        L.collect()
        if i == 0:
            b = L._bufs
            first = {k: b[k].cpu().clone() for k in ("feats", "masks", "actions", "values", "rewards", "term",
                                                       "trunc")}
        L.update()
        L.roll_over()
        if i == 0:
            params1 = flat(L)
    torch.cuda.synchronize()
    torch.save({"first": first, "params1": params1, "params": flat(L), "critic": L.critic_loss_history,
                "actor": [L.actor_loss_history[k] for k in A.AGENTS],
                "exchange_bytes": L.exchange_bytes_per_batch()},
               os.path.join(a.shard_out, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
