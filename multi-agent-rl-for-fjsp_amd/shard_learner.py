"""The A2C update sharded by learner over the ranks of a multi-GPU job (BASELINE config 5,
exchange="shard"): the reference's experience exchange (a2c.py:324-336: memory ->
finish_trajectory -> _update over every transition) routed to the rank that learns from it,
instead of gathered into one rank that learns from all of it.

Reference update (a2c.py:647-731, networks.py:22-61): 8 independent actors, each trained on its
own agent's (observation, mask, action, advantage) samples, and one centralised critic trained on
(global state, returns).  So the learner splits by network:

  * actor a is owned by rank a mod world; the critic's distinct global states are owned by the
    rank their group key hashes to (16 key bits, dealt in proportion to per-rank weights: the AGV
    actor's owner takes half a share), so every distinct state is learned on exactly one rank;
  * each rank first COMBINES its own samples (a combiner in the map-reduce sense): the actor
    loss is linear in the normalised advantage for a fixed (input, mask, action), and the
    critic's loss gradient in the returns for a fixed state, so

      actor record  = (agent, input, mask bits, action, #samples, sum of normalised advantages)
      critic record = (global state, #samples, sum over samples and agents of R, of R^2)

    carry everything the owner needs; a sample's record is found by one flat radix sort of
    hashed keys (RowGroups), checked bit for bit against the group's representative (a hash
    collision makes the whole batch fall back to the all-reduce exchange);
  * ONE all_to_all moves the records to their owners (RCCL over xGMI, point to point: each pair
    of ranks exchanges only what the receiver learns from);
  * every owner merges equal inputs across source ranks, runs its actors / its share of the
    critic once per distinct input, and back-propagates the combined losses;
  * ONE all_reduce of the flat gradient (8 stacked actors + critic, 2.7 MB; each rank contributes
    its own networks' gradients, zeros elsewhere) + the loss partials + the collision flag, then
    the same clipping and Adam step on every rank: the parameters stay identical everywhere, no
    broadcast.

The result equals one learner over all ranks' transitions up to the summation order of the
gradients (tests/test_gpu_config5.py: <= 1e-5 relative per tensor at 8 x 4 096 envs).  The same
functions run without a process group (emulate()) so that one GPU can time every rank's share.
"""
import torch

from . import a2c_vec as A
from . import distributed as D

NA = A.NA
# record layouts, int32 words (8-byte fields first, 8-byte aligned rows)
AW = 20   # actor:  key i64 | sum adv_n f64 | input f32[13] | bits | act << 8 | agent << 16 | count | pad
CW = 46   # critic: key i64 | sum R f64 | sum R^2 f64 | count | pad | global state f32[38]
_MIX = A._s64(0x9E3779B97F4A7C15)


def owner_of_agent(a, world):
    return a % world


# the critic's states are dealt to the ranks by 16 bits of their key in proportion to these
# weights: the rank that owns the AGV's actor (1.2 M of config 5's 1.3 M actor records) takes half
# a share of the critic, so the ranks' learner shares even out
AGV = 1
AGV_CRITIC_SHARE = 0.5


def critic_bounds(world):
    """Upper bucket edges (16-bit hash values) of ranks 0 .. world - 2 for the critic's states."""
    w = [AGV_CRITIC_SHARE if owner_of_agent(AGV, world) == r else 1.0 for r in range(world)]
    tot, acc, out = sum(w), 0.0, []
    for r in range(world - 1):
        acc += w[r]
        out.append(int(round(65536 * acc / tot)))
    return out


# the 16 key bits that pick a critic state's owner: the top 16 of the 59 bits RowGroups sorts by,
# so the grouping's distinct states come out already ordered by owner rank
DEST_SHIFT = 43


def _critic_dest(key, world):
    if world == 1:
        return torch.zeros_like(key)
    b = A._index_tensor(tuple(critic_bounds(world)), key.device)
    return torch.searchsorted(b, (key >> DEST_SHIFT) & 0xFFFF, right=True)


def _group_sums(perm, ends, vals):
    """Per group of a RowGroups row set (perm [R, S], ends [R, U]): the f64 sums of vals [R, S]
    (or [C, S] with R = 1) over each group's samples, in sorted order (prefix sums differenced at
    the run ends, deterministic).  Padding groups (ends = S) sum to 0."""
    C = vals.shape[0]
    if perm.shape[0] == 1 and C > 1:
        perm, ends = perm.expand(C, -1), ends.expand(C, -1)
    ws = torch.gather(vals, 1, perm)
    ce = A._prefix_at(ws, (ends - 1).clamp(min=0))
    return torch.cat([ce[:, :1], ce[:, 1:] - ce[:, :-1]], dim=1)


def _counts(ends):
    starts = torch.cat([torch.zeros_like(ends[:, :1]), ends[:, :-1]], dim=1)
    return ends - starts


def _i32(t, cols):
    """A field as int32 words [U, cols] (bit patterns)."""
    return t.contiguous().view(torch.int32).reshape(-1, cols)


def _verify_rows(rows, rep, cols):
    """True when rows[rep[s], cols] == rows[s, cols] bitwise for every s (CPU path)."""
    r = rows.view(torch.int32)
    return bool((r[rep][:, cols] == r[:, cols]).all())


class Combined:
    """One rank's records, ordered by destination rank: actor [Ra, AW] and critic [Rc, CW] int32,
    counts [world, 2] int64 on the records' device (actor, critic records per destination; the
    host copy comes with the exchange's one synchronisation), bad = 0-d float tensor (1: a hash
    collision or a non-binary mask; the batch must fall back)."""

    def __init__(self, actor, critic, counts, bad, samples):
        self.actor, self.critic, self.counts, self.bad, self.samples = actor, critic, counts, bad, samples
        self._host = None

    @property
    def counts_host(self):
        """[world, 2] int64 on the host (synchronises unless exchange() already fetched it)."""
        if self._host is None:
            self._host = self.counts.cpu()
        return self._host

    def flat(self):
        """The send buffer (int32 words, per destination: its actor records, then its critic
        records) and the split sizes in words."""
        pieces, splits = [], []
        a0 = c0 = 0
        for na, nc in self.counts_host.tolist():
            pieces += [self.actor[a0:a0 + na].reshape(-1), self.critic[c0:c0 + nc].reshape(-1)]
            splits.append(AW * na + CW * nc)
            a0 += na
            c0 += nc
        return torch.cat(pieces), splits

    def bytes_by_dest(self):
        return [4 * (AW * na + CW * nc) for na, nc in self.counts_host.tolist()]


def shard_info_words(masks, actions):
    """Per (agent, sample s = t n + e): the agent's mask bits | its action << 8 (int32 [8, S]) from
    masks int8 [T, 29, n] (0 / 1) and actions u8 [T, 8, n]."""
    T, _, n = masks.shape
    S = T * n
    dev = masks.device
    sh = torch.arange(A.MASK_DIM, dtype=torch.int32, device=dev).view(1, -1, 1)
    bits29 = ((masks != 0).to(torch.int32) << sh).sum(1, dtype=torch.int32).reshape(S)  # [S]
    offs = A._index_tensor(tuple(A.MASK_OFFS), dev).to(torch.int32)
    low = A._index_tensor(tuple((1 << k) - 1 for k in A.N_ACTIONS), dev).to(torch.int32)
    bits = (bits29[None, :] >> offs[:, None]) & low[:, None]                             # [8, S]
    act = actions.permute(1, 0, 2).reshape(NA, S).to(torch.int32)
    return bits | (act << 8)


def combine(feats, masks, actions, ret, adv, mean, std, world):
    """The combiner: this rank's [T, ., n] batch (feats f32 [T, 38, n], masks int8 [T, 29, n],
    actions u8 [T, 8, n], ret / adv f64 [T, 8, n]) -> its actor and critic records, routed.
    mean / std f32 [8]: the global advantage statistics (None: advantages as they are,
    calc_actor_loss with one sample)."""
    T, _, n = feats.shape
    S = T * n
    dev = feats.device
    f3 = feats.contiguous()
    if f3.is_cuda:
        rows = torch.empty(S, A.GROUP_ROW, dtype=torch.float32, device=dev)
        keys = A.group_keys(f3, rows)
    else:
        keys = A.group_keys(f3)
        rows = A.feature_rows(f3)
    m = masks.contiguous()
    if f3.is_cuda:
        # info and record keys in one pass (fjsp_a2c_shard_keys: the torch formula below)
        import ctypes
        tk = torch.empty(NA + 1, S, dtype=torch.int64, device=dev)
        info = torch.empty(NA, S, dtype=torch.int32, device=dev)
        nb = torch.zeros(-(-S // 256), dtype=torch.int32, device=dev)
        V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        A.nat.check(A.nat.lib().fjsp_a2c_shard_keys(V(keys), V(m), V(actions.contiguous()), T, n, V(tk), V(info), V(nb),
                                                    ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
        tk[NA].copy_(keys[NA])
        bad = nb.any()
    else:
        bad = (~((m == 0) | (m == 1))).any()
        info = shard_info_words(m, actions)
        tk = torch.cat([A._fmix64(keys[:NA] ^ A._fmix64(info.to(torch.int64) * _MIX + 1)), keys[NA:]])
    g = A.RowGroups(tk, A.STATION_ROWS)                                                  # 8 + 1 rows
    U = g.U
    # every sample equals its group's representative: the input bitwise, the mask bits and action
    if rows.is_cuda:
        import ctypes
        flag = torch.empty(-(-S // 256), dtype=torch.int32, device=dev)
        V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        A.nat.check(A.nat.lib().fjsp_a2c_group_verify(V(rows), T, n, V(g.rep[:NA].contiguous()),
                                                      V(g.rep[NA].contiguous()), V(flag),
                                                      ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
        bad = bad | flag.any()
    else:
        gidx = A.gather_index(dev)
        ok = all(_verify_rows(rows, g.rep[a], gidx[a]) for a in range(NA))
        ok = ok and _verify_rows(rows, g.rep[NA], torch.arange(A.GLOBAL_DIM))
        bad = bad | torch.tensor(not ok)
    bad = bad | (torch.gather(info, 1, g.rep[:NA]) != info).any()

    # per group: count and f64 sums in sorted order
    adv32 = adv.float().permute(1, 0, 2).reshape(NA, S)
    advn = (adv32 - mean[:, None]) / (std[:, None] + 1e-8) if mean is not None else adv32
    if g.gsorted is not None:   # one run-sum pass (f64 in sorted order, fjsp_a2c_run_sums)
        sadv = A.run_sums(advn, A._index_tensor(tuple(range(NA)), dev), None, g).double()  # [8, Umax]
    else:
        sadv = _group_sums(g.perm[:NA], g.ends[:NA], advn.double())
    if ret.is_cuda:
        rs, _ = A.slab_stats(ret=ret)                                                     # [2, S], one pass
    else:
        r32 = ret.float().double()                                                       # [T, 8, n]
        rs = torch.stack([r32.sum(1).reshape(S), (r32 * r32).sum(1).reshape(S)])
    cs = _group_sums(g.perm[NA:], g.ends[NA:], rs)                                       # [2, Umax]
    cnt = _counts(g.ends).to(torch.int32)                                                # [9, Umax]

    # actor records, built in owner-rank order (each agent's groups in key order)
    agents = [a for d in range(world) for a in range(NA) if owner_of_agent(a, world) == d]
    na_d = [sum(U[a] for a in range(NA) if owner_of_agent(a, world) == d) for d in range(world)]
    ai = torch.cat([torch.full((U[a],), a, dtype=torch.int64, device=dev) for a in agents])
    gi = torch.cat([torch.arange(U[a], device=dev) for a in agents])
    s1 = g.first[ai, gi]
    x = torch.gather(rows.index_select(0, s1), 1, A.gather_index(dev)[ai])               # [Ua, 13]
    word = info[ai, s1] | (ai.to(torch.int32) << 16)
    arec = torch.cat([_i32(keys[ai, s1], 2), _i32(sadv[ai, gi], 2), _i32(x, 13), word[:, None], cnt[ai, gi][:, None],
                      torch.zeros_like(word)[:, None]], dim=1)

    # critic records: the grouping's order is ascending in the 59 sorted key bits, so ascending in
    # the owner bits (DEST_SHIFT) too — already ordered by owner rank
    uc = U[NA]
    s1 = g.first[NA, :uc]
    ck = keys[NA].index_select(0, s1)
    crec = torch.cat([_i32(ck, 2), _i32(cs[0, :uc], 2), _i32(cs[1, :uc], 2), cnt[NA, :uc][:, None],
                      torch.zeros(uc, 1, dtype=torch.int32, device=dev),
                      _i32(rows.index_select(0, s1)[:, :A.GLOBAL_DIM], A.GLOBAL_DIM)], dim=1)
    dest = _critic_dest(ck, world)
    # the records must leave in owner order for the all_to_all's contiguous splits: RowGroups sorts
    # the 59 key bits whose top 16 (DEST_SHIFT) pick the owner, so dest is non-decreasing; a break
    # of that invariant would mis-route records silently, so it raises the collision flag (fallback)
    if uc > 1:
        bad = bad | (dest[1:] < dest[:-1]).any()
    counts = torch.empty(world, 2, dtype=torch.int64, device=dev)
    counts[:, 0].copy_(torch.tensor(na_d, dtype=torch.int64), non_blocking=True)
    counts[:, 1] = torch.bincount(dest, minlength=world)            # on the device: no host sync here
    return Combined(arec, crec, counts, bad.float().reshape(()), S)


def exchange(comb, group):
    """ONE all_to_all of the records (after one of the [world, 2] counts): returns this rank's
    received (actor [Ra, AW], critic [Rc, CW]) records in source-rank order and the bytes this rank
    sent to other ranks."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    gloo = dist.get_backend(group) == "gloo"
    dev = comb.actor.device
    cdev = torch.device("cpu") if gloo else dev
    cnt_in = comb.counts.to(cdev)
    cnt_out = torch.empty_like(cnt_in)
    dist.all_to_all_single(cnt_out, cnt_in, group=group)
    # the update's one count synchronisation: what this rank sends and receives, to the host together
    both = torch.stack([cnt_in, cnt_out]).cpu()
    comb._host = both[0]
    rc = both[1].tolist()
    buf, splits = comb.flat()
    osplits = [AW * na + CW * nc for na, nc in rc]
    src = buf.cpu() if gloo else buf
    out = torch.empty(sum(osplits), dtype=torch.int32, device=cdev)
    dist.all_to_all_single(out, src, output_split_sizes=osplits, input_split_sizes=splits, group=group)
    out = out.to(dev)
    sent = 4 * (sum(splits) - splits[rank])
    return _parse(out, rc), sent


def _parse(out, rc):
    acts, crits, off = [], [], 0
    for na, nc in rc:
        acts.append(out[off:off + AW * na].view(na, AW))
        off += AW * na
        crits.append(out[off:off + CW * nc].view(nc, CW))
        off += CW * nc
    return torch.cat(acts), torch.cat(crits)


def emulate(combs):
    """The all_to_all without a process group (one process holding every rank's Combined, in rank
    order): the records each destination rank would receive."""
    world = len(combs)
    out = []
    for d in range(world):
        acts, crits = [], []
        for c in combs:
            ch = c.counts_host
            a0 = int(ch[:d, 0].sum())
            c0 = int(ch[:d, 1].sum())
            acts.append(c.actor[a0:a0 + int(ch[d, 0])])
            crits.append(c.critic[c0:c0 + int(ch[d, 1])])
        out.append((torch.cat(acts), torch.cat(crits)))
    return out


class _RecordHead(torch.autograd.Function):
    """One agent's actor loss over its records on the GPU (fjsp_a2c_record_head): forward the loss
    and each record's gradient with respect to its input's eight probabilities; backward the
    records' gradients summed per input group (runs of the sorted order, fjsp_a2c_run_sums).
    pu f32 [8, Umax] per distinct input (RowGroups g, one row), info i32 [R], wsum f64 [R], cnt
    i32 [R]."""

    @staticmethod
    def forward(ctx, pu, g, info, wsum, cnt, na, count, coef):
        import ctypes
        R = info.shape[0]
        um = pu.shape[1]
        dev = pu.device
        grad = torch.empty(na, R, dtype=torch.float32, device=dev)
        sums = torch.empty(-(-R // 256), 2, dtype=torch.float64, device=dev)
        pc = pu.detach().contiguous()
        V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        A.nat.check(A.nat.lib().fjsp_a2c_record_head(V(pc), um, V(g.inv[0].contiguous()), R, na, V(info), V(wsum),
                                                     V(cnt), 1.0 / count, float(coef), V(grad), V(sums),
                                                     ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
        s = sums.sum(0)
        ctx.g, ctx.na, ctx.um = g, na, um
        ctx.save_for_backward(grad)
        return ((-s[0] - coef * s[1]) / count).float()

    @staticmethod
    def backward(ctx, gl):
        (grad,) = ctx.saved_tensors
        na, um = ctx.na, ctx.um
        rowmap = torch.zeros(na, dtype=torch.int32, device=grad.device)
        rs = A.run_sums(grad, rowmap, gl.reshape(1).expand(na).float(), ctx.g)                  # [na, Umax]
        out = torch.zeros(8, um, dtype=grad.dtype, device=grad.device)
        out[:na] = rs
        return out, None, None, None, None, None, None, None


def _regroup(key):
    """RowGroups of one row of record keys, or None for no records."""
    if key.numel() == 0:
        return None
    return A.RowGroups(key.reshape(1, -1))


def owner_losses(actors, critic, recv, rank, world, count, entropy_coef):
    """This rank's share of the losses (a2c.py:647-731) from its received records, with the
    autograd graph into its own actors and the critic: (actor losses [8] (zeros for the agents
    other ranks own), critic loss (0-d), bad (0-d float: a collision among the records))."""
    arec, crec = recv
    dev = arec.device
    al = torch.zeros(NA, dtype=torch.float32, device=dev)
    cl = torch.zeros((), dtype=torch.float32, device=dev)
    bad = torch.zeros((), dtype=torch.bool, device=dev)
    mine = [a for a in range(NA) if owner_of_agent(a, world) == rank]
    agent = (arec[:, AW - 3] >> 16) & 0xFF if len(mine) > 1 else None
    for a in mine:
        r = arec if agent is None else arec[agent == a]   # one owned agent: every record is its
        g = _regroup(r[:, 0:2].contiguous().view(torch.int64).reshape(-1))
        if g is None:
            continue
        # equal keys must mean equal inputs (bitwise), across source ranks too
        xi = r[:, 4:4 + A.DPAD]
        bad = bad | (xi.index_select(0, g.rep[0]) != xi).any()
        u = g.U[0]
        xu = xi.index_select(0, g.first[0, :u]).contiguous().view(torch.float32)          # [u, 13]
        pu = actors.agent_probs(a, xu.t())                                                # [8, u]
        um = g.first.shape[1]
        if um > u:
            pu = torch.nn.functional.pad(pu, (0, um - u))
        info = r[:, AW - 3]
        k = A.N_ACTIONS[a]
        if r.is_cuda and g.gsorted is not None:
            la = _RecordHead.apply(pu, g, info.contiguous(), r[:, 2:4].contiguous().view(torch.float64).reshape(-1),
                                   r[:, AW - 2].contiguous(), k, count, entropy_coef)
            al = al + torch.nn.functional.one_hot(torch.tensor(a, device=dev), NA).float() * la
            continue
        p = g.gather(pu[None])                                                            # [1, 8, R]
        j = torch.arange(8, device=dev, dtype=torch.int32)
        m = (((info[None, :] >> j[:, None]) & 1) * (j[:, None] < k)).to(torch.float32)[None]  # [1, 8, R]
        act = ((info >> 8) & 0xFF).long()[None]
        w = r[:, 2:4].contiguous().view(torch.float64).reshape(-1).float()
        nrec = r[:, AW - 2].float()
        ent = A.entropy_of(p)[0]
        logp = A.categorical_log_prob(A.masked_probs(p, m), act)[0]
        la = -(w * logp).sum() / count - entropy_coef * (nrec * ent).sum() / count
        al = al + torch.nn.functional.one_hot(torch.tensor(a, device=dev), NA).float() * la
    g = _regroup(crec[:, 0:2].contiguous().view(torch.int64).reshape(-1))
    if g is not None and crec.is_cuda and A.critic_fused and A.critic_onepass_on and g.gsorted is not None:
        # the critic's share in one pass per distinct state (fjsp_a2c_critic_fused): the records of
        # one state (from every source rank) merged into its sample count and return sums
        xs = crec[:, 8:8 + A.GLOBAL_DIM]
        bad = bad | (xs.index_select(0, g.rep[0]) != xs).any()
        vals = torch.stack([crec[:, 6].double(), crec[:, 2:4].contiguous().view(torch.float64).reshape(-1),
                            crec[:, 4:6].contiguous().view(torch.float64).reshape(-1)])
        su = _group_sums(g.perm, g.ends, vals)                                            # [3, Umax]
        x = torch.nn.functional.pad(xs.index_select(0, g.first[0]).contiguous().view(torch.float32),
                                    (0, A.GROUP_ROW - A.GLOBAL_DIM))                     # [Umax, 40]
        cl = A.critic_onepass(critic, x, A.critic_coef_sums(su[0], su[1], su[2], count))
    elif g is not None:
        xs = crec[:, 8:8 + A.GLOBAL_DIM]
        bad = bad | (xs.index_select(0, g.rep[0]) != xs).any()
        u = g.U[0]
        x = torch.nn.functional.pad(xs.index_select(0, g.first[0, :u]).contiguous().view(torch.float32),
                                    (0, A.GROUP_ROW - A.GLOBAL_DIM))                     # [u, 40]
        if x.is_cuda and u >= 65536 and A.critic_fused:
            vu = A.critic_grouped(critic, x)
        else:
            vu = A.mlp_forward(critic.net, x[:, :A.GLOBAL_DIM]).reshape(-1)
        um = g.first.shape[1]
        vu = torch.nn.functional.pad(vu.reshape(1, 1, -1), (0, um - u))
        v = g.gather(vu).reshape(-1).double()                                             # [Rc]
        nrec = crec[:, 6].double()
        sr = crec[:, 2:4].contiguous().view(torch.float64).reshape(-1)
        sr2 = crec[:, 4:6].contiguous().view(torch.float64).reshape(-1)
        # sum over the group's samples and agents of (V - R)^2, expanded
        cl = ((NA * nrec * v * v - 2.0 * v * sr + sr2).sum() / (NA * count)).float()
    return al, cl, bad.float()


def _params(actors, critic):
    return list(actors.parameters()) + list(critic.parameters())


def reduce_grads(actors, critic, al, cl, bad, group):
    """ONE all_reduce (sum) of [every gradient | actor losses | critic loss | bad]; the summed
    gradients are written back (created where a rank had none).  Returns (al, cl, bad) summed."""
    import torch.distributed as dist
    ps = _params(actors, critic)
    flat = torch.cat([A.flat_grads(actors, critic), al.detach().float(), cl.detach().float().reshape(1),
                      bad.reshape(1)])
    if group is not None:
        gloo = dist.get_backend(group) == "gloo"
        buf = flat.cpu() if gloo else flat
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        flat = buf.to(flat.device)
    off = 0
    for p in ps:
        k = p.numel()
        g = flat[off:off + k].view_as(p)
        if p.grad is None:
            p.grad = g.clone()
        else:
            p.grad.copy_(g)
        off += k
    return flat[off:off + NA], flat[off + NA], flat[off + NA + 1]


def update_sharded(actors, critic, optim_actor, optim_critic, feats, masks, actions, ret, adv, gidx, midx,
                   entropy_coef, max_grad_norm, group, dedup=True, grad_probe=None, info=None, stage=None):
    """One _update (a2c.py:647-703) over every rank's transitions with the learner sharded by
    network (module docstring).  Collective calls, in order: the advantage statistics
    (all_reduce), the record counts and the records (all_to_all), the gradients + losses + flag
    (all_reduce).  Host synchronisations: the advantage count, the record counts (one, for both
    directions) and the reduced losses + flag (one).  info (dict): filled with this rank's record
    counts and bytes sent.  stage (callable(name) or None): called at the end of each stage
    (adv_stats, combine, exchange, own, all_reduce, clip_adam) by the bench's synchronised stage
    timer.  Returns (actor losses [8], critic loss) as Python floats."""
    import torch.distributed as dist
    mark = stage if stage is not None else (lambda name: None)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    count, mean, std = D.adv_stats_slab(adv, group)
    norm = count > 1
    mark("adv_stats")
    comb = combine(feats, masks, actions, ret, adv, mean if norm else None, std if norm else None, world)
    mark("combine")
    recv, sent = exchange(comb, group)
    mark("exchange")
    optim_actor.zero_grad(set_to_none=True)
    optim_critic.zero_grad(set_to_none=True)
    al, cl, bad = owner_losses(actors, critic, recv, rank, world, count, entropy_coef)
    bad = torch.maximum(bad, comb.bad)
    if al.requires_grad or cl.requires_grad:
        (al.sum() + cl).backward()
    mark("own")
    al, cl, bad = reduce_grads(actors, critic, al, cl, bad, group)
    tail = torch.cat([al.float(), cl.float().reshape(1), bad.float().reshape(1)]).cpu().tolist()   # one sync
    mark("all_reduce")
    if info is not None:
        ch = comb.counts_host
        info.update({"actor_records_sent": int(ch[:, 0].sum()), "critic_records_sent": int(ch[:, 1].sum()),
                     "actor_records_received": int(recv[0].shape[0]), "critic_records_received": int(recv[1].shape[0]),
                     "samples": comb.samples, "bytes_sent_to_other_ranks": sent,
                     "bytes_by_dest": comb.bytes_by_dest(), "fallback": tail[NA + 1] > 0})
    if tail[NA + 1] > 0:
        # a hash collision somewhere (or a non-binary mask, or records out of owner order): the
        # all-reduce exchange's update, which checks its own grouping and falls back to the dense
        # update if needed
        al2, cl2 = A.update_core(actors, critic, optim_actor, optim_critic, feats, masks, actions, ret, adv, gidx,
                                 midx, entropy_coef, max_grad_norm, group, dedup, grad_probe)
        return al2.cpu().tolist(), float(cl2.cpu()[0])
    if grad_probe is not None:
        grad_probe(A.flat_grads(actors, critic).detach().clone())
    A.clip_per_agent_(actors, max_grad_norm)
    torch.nn.utils.clip_grad_norm_(critic.parameters(), max_grad_norm)
    optim_actor.step()
    optim_critic.step()
    mark("clip_adam")
    return tail[:NA], tail[NA]
