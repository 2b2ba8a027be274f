"""Multi-GPU plumbing: one process per GPU, envs sharded by global id.

Stepping needs no collective: rank r owns global env ids [r*n, (r+1)*n) and every result
depends only on (seed, global id, action stream), so shards are bit-identical to the same envs
on one GPU.  The only exchange is once per A2C batch:

  * default: every rank computes GAE locally and its share of the loss sums, then ONE bucketed
    all_reduce of the flattened gradients (8 stacked actors + critic, ~2.7 MB f32) plus two
    tiny all_reduces of advantage statistics -> the update equals a single learner's over all
    ranks' transitions.  On xGMI (point-to-point links) one 2.7 MB ring all_reduce per batch is
    per-link bound and costs well under a millisecond;
  * gather_transitions: the §8(e) alternative — all_gather of a rank's transition slab into
    a learner-side [world, ...] tensor (e.g. to feed an external learner).

The torch.distributed backend is "nccl" (= RCCL on ROCm) on GPUs and "gloo" in CPU tests.
"""
import os

import torch
import torch.distributed as dist


def active(group=None):
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


def rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def shard_range(envs_per_rank, rank):
    """Global env ids owned by `rank` (env_id_base, count)."""
    return rank * envs_per_rank, envs_per_rank


def init_from_env(backend=None):
    """init_process_group from torchrun's environment (RANK / WORLD_SIZE / MASTER_ADDR ...);
    returns (rank, world, local_rank).  No-op for a single process."""
    world = int(os.environ.get("WORLD_SIZE", 1))
    rank = int(os.environ.get("RANK", 0))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        dist.init_process_group(backend=backend)
    return rank, world, local


def allreduce_sum(t, group=None):
    if active(group):
        t = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def allreduce_max(t, group=None):
    if active(group):
        t = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t


def adv_stats(adv, group=None):
    """Global per-agent count, mean and unbiased std of advantages adv [A, S_local] (f32).

    Single process: exactly Tensor.mean / Tensor.std as calc_actor_loss (a2c.py:724-731).
    Sharded: f64 sums of x and x^2 over all ranks."""
    if not active(group):
        return adv.shape[1], adv.mean(dim=1), adv.std(dim=1)
    x = adv.double()
    s = torch.stack([x.sum(dim=1), (x * x).sum(dim=1),
                     torch.full_like(x[:, 0], float(adv.shape[1]))], dim=1)
    dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
    n = s[0, 2]
    mean = s[:, 0] / n
    var = (s[:, 1] - n * mean * mean) / (n - 1)
    return int(n.item()), mean.float(), var.clamp_min(0).sqrt().float()


def allreduce_grads(params, group=None):
    """Sum every parameter's gradient over ranks with ONE flat bucket (one RCCL ring pass)."""
    if not active(group):
        return
    grads = [p.grad for p in params if p.grad is not None]
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


def gather_transitions(slab, group=None):
    """all_gather of equally shaped per-rank transition slabs -> [world, *slab.shape]."""
    if not active(group):
        return slab.unsqueeze(0)
    world = dist.get_world_size(group)
    flat = slab.contiguous().reshape(-1)
    out = torch.empty(world * flat.numel(), dtype=slab.dtype, device=slab.device)
    dist.all_gather_into_tensor(out, flat, group=group)
    return out.view((world,) + tuple(slab.shape))


def broadcast_params(module, src=0, group=None):
    """Make every rank start from rank src's parameters."""
    if not active(group):
        return
    for p in module.parameters():
        dist.broadcast(p.data, src=src, group=group)
