#!/usr/bin/env python3
"""The critic's weight gradients gy^T x over U distinct states: the f32 split-K batched GEMM
(a2c_vec._splitk_wgrad, today) against the same split-K on bf16 planes (hi, mid of each f32
operand; hi.hi + hi.mid + mid.hi, f32 accumulate via bmm(out_dtype=float32)), with the planes
given (as the fused critic kernel could write them in place of the f32 values).  Times per GEMM
(CUDA events, median of 20) and the error of each against float64.

usage: python scripts/ab_wgrad_planes.py [U]"""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")


def planes(x):
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


def splitk_planes(gp, xp, c=128):
    """sum over (hi.hi, hi.mid, mid.hi) of the split-K bmm of bf16 planes, f32 out."""
    gh, gm = gp
    xh, xm = xp
    B = gh.shape[0]
    bc = B // c
    out = None
    for a, b in ((gh, xh), (gh, xm), (gm, xh)):
        ac = a[:c * bc].reshape(c, bc, -1).transpose(1, 2)
        bb = b[:c * bc].reshape(c, bc, -1)
        r = torch.bmm(ac, bb, out_dtype=torch.float32).sum(0)
        if c * bc < B:
            r += torch.mm(a[c * bc:].t(), b[c * bc:], out_dtype=torch.float32)
        out = r if out is None else out + r
    return out


def timed(fn, reps=20):
    ts = []
    for _ in range(reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[3:])
    return ts[len(ts) // 2]


def main(U):
    torch.manual_seed(0)
    dev = "cuda"
    res = {"U": U}
    shapes = {"W2": (256, 256), "W3": (128, 256), "W1": (256, 38)}
    for name, (m, k) in shapes.items():
        g = torch.randn(U, m, device=dev) * (torch.rand(U, m, device=dev) > 0.5)
        x = torch.relu(torch.randn(U, k, device=dev)) if name != "W1" else torch.rand(U, k, device=dev) * 20
        ref = (g.double().t() @ x.double())
        f32 = A._splitk_wgrad(g, x)
        gp, xp = planes(g), planes(x)
        bfp = splitk_planes(gp, xp)
        err = lambda a: float((a.double() - ref).norm() / ref.norm())  # noqa: E731
        res[name] = {"f32_ms": timed(lambda: A._splitk_wgrad(g, x)), "planes_ms": timed(lambda: splitk_planes(gp, xp)),
                     "split_ms": timed(lambda: (planes(g), planes(x))),
                     "f32_rel_err": err(f32), "planes_rel_err": err(bfp)}
        print(name, res[name], flush=True)
    return res


if __name__ == "__main__":
    U = int(sys.argv[1]) if len(sys.argv) > 1 else 540000
    print(json.dumps(main(U)))
