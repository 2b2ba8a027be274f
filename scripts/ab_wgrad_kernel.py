"""A/B of the critic's weight gradients at a full update's distinct-state count: fjsp_a2c_wgrad
(a2c_vec.critic_wgrad, r06) against the split-K hipBLASLt f32 GEMMs (a2c_vec._splitk_wgrad), per
layer, HIP-event time of 20 launches after 3 warm-up ones, and the error of each against float64.
usage: python scripts/ab_wgrad_kernel.py [U] [parts]"""
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
U = int(sys.argv[1]) if len(sys.argv) > 1 else 540000
PARTS = int(sys.argv[2]) if len(sys.argv) > 2 else None
torch.manual_seed(0)


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {"U": U, "parts": PARTS}
tot = [0.0, 0.0]
for name, m, nx, nout in (("W2", 256, 256, 256), ("W3", 128, 256, 256), ("W1", 256, 40, 38)):
    g = torch.randn(U, m, device="cuda") * (torch.rand(U, m, device="cuda") > 0.5)
    x = torch.relu(torch.randn(U, nx, device="cuda"))
    ref = g.double().t() @ x[:, :nout].double()
    k = lambda: A.critic_wgrad(g, x, nout, PARTS)  # noqa: E731
    s = lambda: A._splitk_wgrad(g, x[:, :nout])  # noqa: E731
    err = lambda t: float((t.double() - ref).norm() / ref.norm())  # noqa: E731
    tk, ts = timed(k), timed(s)
    tot[0] += tk
    tot[1] += ts
    res[name] = {"kernel_ms": tk, "splitk_ms": ts, "kernel_err": err(k()), "splitk_err": err(s()),
                 "kernel_GBs": (U * (m + nx) * 4) / tk / 1e6, "kernel_TFs_f32": 2 * U * m * nout / tk / 1e9}
    del g, x, ref
res["total"] = {"kernel_ms": tot[0], "splitk_ms": tot[1]}
print(json.dumps(res, indent=1))
