#!/usr/bin/env python3
"""The gather learner's unpacking of the gathered slabs (distributed.gather_slabs + the
[world, ..., n] -> [..., world * n] view of a2c_vec._update_gathered) at config 5 (8 x 4 096 envs,
256 steps), r04's form against HEAD's, on one GPU: r04 received into 8 buffers, stacked them
([world, bytes] copy), made each tensor contiguous (a second copy) and concatenated the ranks
(a third); HEAD receives into one preallocated [world, bytes] buffer, takes each tensor as a view
and keeps only the concatenation.  Same bytes out (checked).  Prints JSON (ms, medians)."""
import json
import time

import torch

W, T, n = 8, 256, 4096
SLAB = {"feats": ((T, 38, n), torch.float32), "masks": ((T, 29, n), torch.int8), "actions": ((T, 8, n), torch.uint8),
        "rewards": ((T, 8, n), torch.float64), "values": ((T + 1, n), torch.float32), "done": ((T, n), torch.uint8)}


def nbytes(shape, dt):
    k = 1
    for s in shape:
        k *= s
    return k * torch.empty((), dtype=dt).element_size()


def cat(x):
    return x.movedim(0, -2).reshape(*x.shape[1:-1], -1)


def old(bufs):
    allb = torch.stack(bufs)
    out, off = {}, 0
    for k, (shape, dt) in SLAB.items():
        nb = nbytes(shape, dt)
        out[k] = cat(allb[:, off:off + nb].contiguous().view(dt).view((W,) + shape))
        off += nb
    return out


def new(allb, order):
    out, off = {}, 0
    for k in order:
        shape, dt = SLAB[k]
        nb = nbytes(shape, dt)
        out[k] = cat(allb[:, off:off + nb].view(dt).view((W,) + shape))
        off += -(-nb // 8) * 8
    return out


def timed(fn, reps=7):
    ms = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o = fn()
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
        del o
    return sorted(ms)[reps // 2]


def main():
    dev = torch.device("cuda", 0)
    order = sorted(SLAB, key=lambda k: -torch.empty((), dtype=SLAB[k][1]).element_size())
    tot_old = sum(nbytes(*SLAB[k]) for k in SLAB)
    tot_new = sum(-(-nbytes(*SLAB[k]) // 8) * 8 for k in order)
    g = torch.Generator(device=dev).manual_seed(0)
    allb = torch.randint(0, 256, (W, tot_new), dtype=torch.uint8, device=dev, generator=g)
    # the same payload in r04's packing (names in slab order, no padding)
    bufs = []
    for w in range(W):
        parts, off = {}, 0
        for k in order:
            nb = nbytes(*SLAB[k])
            parts[k] = allb[w, off:off + nb]
            off += -(-nb // 8) * 8
        bufs.append(torch.cat([parts[k] for k in SLAB]))
    a, b = old(bufs), new(allb, order)
    same = all(torch.equal(a[k].contiguous().view(torch.uint8), b[k].contiguous().view(torch.uint8)) for k in SLAB)
    del a, b
    res = {"world": W, "steps": T, "envs_per_rank": n, "gathered_bytes": W * tot_old, "outputs_equal": same,
           "r04_unpack_ms": timed(lambda: old(bufs)), "head_unpack_ms": timed(lambda: new(allb, order))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
