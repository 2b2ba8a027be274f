"""A/B of fjsp_a2c_wgrad's 8-wave and 16-wave kernels (library-wide option "wgrad_waves") for the
critic's three layer shapes at U distinct states: HIP-event time of 20 calls (two alternating
rounds), error against float64, and bit-equality of the two.  usage: python scripts/ab_wgrad_waves.py [U]"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
U = int(sys.argv[1]) if len(sys.argv) > 1 else 540000
torch.manual_seed(0)
res = {"U": U}
for name, m, nx, nout in (("W2", 256, 256, 256), ("W3", 128, 256, 256), ("W1", 256, 40, 38)):
    g = torch.randn(U, m, device="cuda") * (torch.rand(U, m, device="cuda") > 0.5)
    x = torch.relu(torch.randn(U, nx, device="cuda"))
    ref = g.double().t() @ x[:, :nout].double()
    r, outs = {}, {}
    for w in (8, 16, 8, 16):
        assert A.nat.lib().fjsp_set_option(None, b"wgrad_waves", w) == 0
        for _ in range(3):
            A.critic_wgrad(g, x, nout)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            o = A.critic_wgrad(g, x, nout)
        e1.record()
        torch.cuda.synchronize()
        r.setdefault(f"ms_{w}", []).append(e0.elapsed_time(e1) / 20)
        outs[w] = o
        r[f"err_{w}"] = float((o.double() - ref).norm() / ref.norm())
    r["bit_equal"] = bool(torch.equal(outs[8], outs[16]))
    res[name] = r
    del g, x, ref
A.nat.lib().fjsp_set_option(None, b"wgrad_waves", 16)
print(json.dumps(res, indent=1))
