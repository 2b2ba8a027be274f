"""Multi-GPU plumbing: one process per GPU, envs sharded by global id.

Stepping needs no collective: rank r owns global env ids [r*n, (r+1)*n) and every result
depends only on (seed, global id, action stream), so shards are bit-identical to the same envs
on one GPU.  The only exchange is once per A2C batch:

  * default: every rank computes GAE locally and its share of the loss sums, then ONE bucketed
    all_reduce of the flattened gradients (8 stacked actors + critic, ~2.7 MB f32) plus two
    tiny all_reduces of advantage statistics -> the update equals a single learner's over all
    ranks' transitions.  On xGMI (point-to-point links) one 2.7 MB ring all_reduce per batch is
    per-link bound and costs well under a millisecond;
  * exchange="gather" (VecMultiAgentA2C): the north star's experience gather — every rank's
    transition slab (features, masks, actions, rewards, values, episode ends; ~258 B per
    env-step) is gathered into the learner rank in ONE collective (gather_slabs), the learner
    runs GAE + the update over the whole batch exactly as a single learner would, and ONE flat
    broadcast (broadcast_flat) hands the new parameters (and the loss values) back;
  * gather_transitions: all_gather of a rank's transition slab into a [world, ...] tensor on
    every rank (e.g. to feed an external learner).

The torch.distributed backend is "nccl" (= RCCL on ROCm) on GPUs and "gloo" in CPU tests.
"""
import os

import torch
import torch.distributed as dist


LOCAL = "local"   # group argument meaning "this process only" (no collective, even when initialised)
# tests: treat an initialised single-rank group as active, so that the collective code paths (the
# device-tensor branches under RCCL) run on one GPU
FORCE_ACTIVE = False


def active(group=None):
    if group is LOCAL:
        return False
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return FORCE_ACTIVE or dist.get_world_size(group) > 1


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


def max_over_ranks(value, group=None, device=None):
    """max of a non-negative Python int over the ranks (the value itself without a group): RCCL
    reduces a device tensor, gloo a host one."""
    if not active(group):
        return value
    dev = torch.device("cpu") if _backend(group) == "gloo" else (device or torch.device("cuda", torch.cuda.current_device()))
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def adv_stats(adv, group=None):
    """Global per-agent count, mean and unbiased std of advantages adv [A, S_local] (f32).

    Single process: exactly Tensor.mean / Tensor.std as calc_actor_loss (a2c.py:724-731).
    Sharded: f64 sums of x and x^2 over all ranks."""
    if not active(group):
        if not adv.is_cuda or adv.shape[1] < 65536:
            return adv.shape[1], adv.mean(dim=1), adv.std(dim=1)
        # a few very long rows: f64 sums in blocks of 1024 (a reduction over 8 rows of 10^6
        # keeps most of the chip idle), var = (sum x^2 - n mean^2) / (n - 1)
        n = adv.shape[1]
        x = torch.nn.functional.pad(adv.double(), (0, -n % 1024)).view(adv.shape[0], -1, 1024)
        mean = x.sum(-1).sum(-1) / n
        var = ((x * x).sum(-1).sum(-1) - n * mean * mean) / (n - 1)
        return n, mean.float(), var.clamp_min(0).sqrt().float()
    x = adv.double()
    s = torch.stack([x.sum(dim=1), (x * x).sum(dim=1),
                     torch.full_like(x[:, 0], float(adv.shape[1]))], dim=1)
    dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
    n = s[0, 2]
    mean = s[:, 0] / n
    var = (s[:, 1] - n * mean * mean) / (n - 1)
    return int(n.item()), mean.float(), var.clamp_min(0).sqrt().float()


def adv_stats_slab(adv, group=None):
    """adv_stats of the rollout slab's advantages adv f64 [T, A, N] (their f32 values, as
    calc_actor_loss's FloatTensor(adv)) without an [A, T * N] copy of a long batch: f64 sums over
    the T and N axes (single process, short batches: Tensor.mean / Tensor.std as before)."""
    T, A, N = adv.shape
    if not active(group) and (not adv.is_cuda or T * N < 65536):
        return adv_stats(adv.float().permute(1, 0, 2).reshape(A, T * N), group)
    if adv.is_cuda and A == 8:
        from .a2c_vec import slab_stats
        _, sums = slab_stats(adv=adv)                                                     # one pass
        s = torch.cat([sums, torch.full((A, 1), float(T * N), dtype=torch.float64, device=adv.device)], dim=1)
    else:
        x = adv.float().double()
        s = torch.stack([x.sum(dim=(0, 2)), (x * x).sum(dim=(0, 2)),
                         torch.full((A,), float(T * N), dtype=torch.float64, device=adv.device)], dim=1)
    if active(group):
        dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
        count = int(s[0, 2].item())                      # every rank's samples (one host sync)
    else:
        count = T * N                                    # known here: no host sync
    n = s[0, 2]
    mean = s[:, 0] / n
    var = (s[:, 1] - n * mean * mean) / (n - 1)
    return count, mean.float(), var.clamp_min(0).sqrt().float()


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


def _backend(group=None):
    return dist.get_backend(group) if active(group) else None


def gather_slabs(slabs, dst=0, group=None):
    """Gather a dict of per-rank tensors (same shapes on every rank) into rank `dst` with ONE
    collective: every tensor is viewed as bytes and packed into one flat buffer.  Returns on
    `dst` a dict of [world, *shape] tensors, None on the other ranks (single process: the
    slabs with a leading axis of 1)."""
    # widest elements first, every piece padded to 8 bytes: each tensor's bytes start 8-byte
    # aligned in the flat buffer, so the results are views of the receive buffer (no copies)
    names = sorted(slabs, key=lambda k: -slabs[k].element_size())
    if not active(group):
        return {k: slabs[k].unsqueeze(0) for k in slabs}
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    pieces = []
    for k in names:
        b = slabs[k].contiguous().view(-1).view(torch.uint8)
        pieces.append(b)
        if b.numel() % 8:
            pieces.append(b.new_zeros(8 - b.numel() % 8))
    flat = torch.cat(pieces)
    gloo = _backend(group) == "gloo"
    src = flat.cpu() if gloo else flat     # gloo gathers host tensors
    allb = bufs = None
    if rank == dst:
        # one preallocated [world, bytes] receive buffer; the gather writes its rows in place
        allb = torch.empty((world, flat.numel()), dtype=torch.uint8, device=src.device)
        bufs = list(allb.unbind(0))
    dist.gather(src, gather_list=bufs, dst=dst, group=group)
    if rank != dst:
        return None
    allb = allb.to(flat.device)
    out, off = {}, 0
    for k in names:
        t = slabs[k]
        nb = t.numel() * t.element_size()
        out[k] = allb[:, off:off + nb].view(t.dtype).view((world,) + tuple(t.shape))   # a strided view
        off += -(-nb // 8) * 8
    return {k: out[k] for k in slabs}


def broadcast_flat(tensors, src=0, group=None):
    """Broadcast a list of tensors from `src` with ONE flat f32 bucket (in place)."""
    if not active(group):
        return
    flat = torch.cat([t.detach().reshape(-1).to(torch.float32) for t in tensors])
    gloo = _backend(group) == "gloo"
    buf = flat.cpu() if gloo else flat
    dist.broadcast(buf, src=src, group=group)
    buf = buf.to(flat.device)
    off = 0
    with torch.no_grad():
        for t in tensors:
            n = t.numel()
            t.copy_(buf[off:off + n].view_as(t).to(t.dtype))
            off += n


def broadcast_params(module, src=0, group=None):
    """Make every rank start from rank src's parameters."""
    if not active(group):
        return
    for p in module.parameters():
        dist.broadcast(p.data, src=src, group=group)
