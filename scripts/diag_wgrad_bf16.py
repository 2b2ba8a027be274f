#!/usr/bin/env python3
"""The critic's weight gradients gW = g^T x over ~5.4 x 10^5 distinct states (diagnostic): the
current f32 split-K batched GEMM (a2c_vec._splitk_wgrad, hipBLASLt f32) against the same sum with
both operands as three bf16 planes (the policy kernel's split arithmetic: six plane products),
as ONE bf16 batched GEMM with f32 output (torch.bmm(..., out_dtype=float32)) over the chunks x
six products.  Times (HIP events, medians) and errors against float64.  Prints JSON."""
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
    r = x - hi.float()
    mid = r.to(torch.bfloat16)
    return hi, mid, (r - mid.float()).to(torch.bfloat16)


def operands(g, x):
    B = x.shape[0]
    c = max(1, min(64, B // 8192))
    bc = B // c
    gp, xp = planes(g[:c * bc]), planes(x[:c * bc])
    pairs = ((0, 0), (0, 1), (1, 0), (1, 1), (0, 2), (2, 0))
    ga = torch.stack([gp[p].reshape(c, bc, -1) for p, _ in pairs]).reshape(6 * c, bc, -1)
    xa = torch.stack([xp[q].reshape(c, bc, -1) for _, q in pairs]).reshape(6 * c, bc, -1)
    return ga, xa, c * bc


def gemm(g, x, ga, xa, n0):
    gW = torch.bmm(ga.transpose(1, 2), xa, out_dtype=torch.float32).sum(0)
    if n0 < x.shape[0]:
        gW += g[n0:].t() @ x[n0:]
    return gW


def wgrad_bf16(g, x):
    return gemm(g, x, *operands(g, x))


def timed(f, reps=10):
    s = torch.cuda.current_stream()
    for _ in range(2):
        f()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        f()
        b.record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2] * 1e3


def main():
    torch.manual_seed(0)
    U = 540097
    out = {"U": U}
    for name, (m, n) in {"W2": (256, 256), "W3": (128, 256), "W1": (256, 38)}.items():
        g = torch.randn(U, m, device="cuda") * (torch.rand(U, m, device="cuda") > 0.5)
        x = torch.relu(torch.randn(U, n, device="cuda"))
        ref = g.double().t() @ x.double()
        a = A._splitk_wgrad(g, x)
        try:
            b = wgrad_bf16(g, x)
            eb = float((b.double() - ref).norm() / ref.norm())
            tb = timed(lambda: wgrad_bf16(g, x))
            tp = timed(lambda: (planes(g), planes(x)))
            ops = operands(g, x)
            tg = timed(lambda: gemm(g, x, *ops))
        except Exception as e:   # out_dtype unsupported on this build
            eb, tb, tp, tg = repr(e)[:200], None, None, None
        out[name] = {"f32_splitk_us": timed(lambda: A._splitk_wgrad(g, x)),
                     "bf16x3_us": tb, "split_planes_us": tp, "bf16x3_gemm_only_us": tg,
                     "err_f32": float((a.double() - ref).norm() / ref.norm()), "err_bf16x3": eb}
        print(json.dumps({name: out[name]}), flush=True)


if __name__ == "__main__":
    main()
