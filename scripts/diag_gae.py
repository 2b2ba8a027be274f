#!/usr/bin/env python3
"""GAE kernel A/B (diagnostic): the r03 kernel against the software-pipelined kernel at several
load-batch depths (build/libgae_ab.so from scripts/diag/gae_ab.hip) and the product library's
fjsp_gae / fjsp_gae_shared.  Outputs are checked bit-equal to the r03 kernel's.  Prints JSON."""
import ctypes
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
L = nat.lib()
AB = ctypes.CDLL(os.path.join(REPO, "build", "libgae_ab.so"))
P, I, D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_double
GEN = [P, P, P, P, I, I, I, D, D, P, P, P]
SH = [P, P, P, I, I, I, D, D, P, P, P]


def fn(lib, name, args):
    f = getattr(lib, name)
    f.restype, f.argtypes = I, args
    return f


def run(T, N, A=8, reps=20):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    M = A * N
    r = (torch.randn(T, M, device=dev, generator=g, dtype=torch.float64) * 24).round() / 8
    v1 = torch.randn(T + 1, N, device=dev, generator=g)
    d = (torch.rand(T, N, device=dev, generator=g) < 0.01).to(torch.uint8)
    vx = v1[:T, None, :].expand(T, A, N).reshape(T, M).contiguous()
    boot = v1[T].double()[None].expand(A, N).reshape(-1).contiguous()
    s = torch.cuda.current_stream(dev)
    V = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    res, ref = {}, None
    cases = [("r03", fn(AB, "gae_r03", GEN), False)]
    for u in (4, 8, 16, 24, 32):
        cases.append((f"u{u}", fn(AB, f"gae_u{u}", GEN), False))
        cases.append((f"shared_u{u}", fn(AB, f"gae_shared_u{u}", SH), True))
    for u, l in ((16, 2), (16, 3), (16, 4), (32, 2)):
        cases.append((f"shared_lw_u{u}_l{l}", fn(AB, f"gae_shared_lw_u{u}_l{l}", SH), True))
    cases.append(("lib_gae", L.fjsp_gae, False))
    cases.append(("lib_gae_shared", L.fjsp_gae_shared, True))
    for name, f, shared in cases:
        ret, adv = torch.empty_like(r), torch.empty_like(r)

        def call():
            if shared:
                rc = f(V(r), V(v1), V(d), T, N, A, 0.99, 0.95, V(ret), V(adv), ctypes.c_void_p(s.cuda_stream))
            else:
                rc = f(V(r), V(vx), V(d), V(boot), T, N, M, 0.99, 0.95, V(ret), V(adv), ctypes.c_void_p(s.cuda_stream))
            assert rc == 0, name
        for _ in range(3):
            call()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(s)
            call()
            b.record(s)
        torch.cuda.synchronize()
        us = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
        if ref is None:
            ref = (ret.clone(), adv.clone())
        eq = bool(torch.equal(ret, ref[0]) and torch.equal(adv, ref[1]))
        # algorithmic bytes: r 8 + ret 8 + adv 8 per element, values 4 per element (generic) or per
        # env-step (shared), done 1 per env-step
        byts = T * M * 24 + (T * M * 4 if not shared else (T + 1) * N * 4) + T * N
        res[name] = {"us_median": us[len(us) // 2], "us_min": us[0], "bit_equal_r03": eq,
                     "algo_bytes": byts, "GBs_median": byts / (us[len(us) // 2] * 1e-6) / 1e9}
    return res


if __name__ == "__main__":
    out = {}
    for T, N in ((256, 4096), (256, 32768), (37, 4096)):
        out[f"T{T}_N{N}"] = run(T, N)
        print(json.dumps({f"T{T}_N{N}": out[f"T{T}_N{N}"]}), flush=True)
