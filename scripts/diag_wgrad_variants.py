"""Which part bounds the critic weight-gradient kernel: time fjsp_a2c_wgrad (W2 / W3 / W1 shapes at U
states) from diagnostic builds of fjsp_policy.hip (scripts/diag/libwg<m>.so, -DWGD=m: 0 as shipped,
1 no loads in the stage loop, 2 no MFMAs, 3 no split / LDS stores).  usage:
python scripts/diag_wgrad_variants.py [U]"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
U = int(sys.argv[1]) if len(sys.argv) > 1 else 540000
res = {"U": U}
P = 256
for mode in range(4):
    L = ctypes.CDLL(os.path.join(REPO, "scripts", "diag", f"libwg{mode}.so"), mode=os.RTLD_LAZY | os.RTLD_LOCAL)
    f = L.fjsp_a2c_wgrad
    f.restype = ctypes.c_int32
    I64, I, V = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
    f.argtypes = [V, I, I64, V, I, I64, I64, V, I, V, I, I64, V]
    r = {}
    for name, m, nx, nout in (("W2", 256, 256, 256), ("W3", 128, 256, 256), ("W1", 256, 40, 38)):
        g = torch.randn(U, m, device="cuda")
        x = torch.randn(U, nx, device="cuda")
        part = torch.empty(P, m, 256 if nx > 64 else 64, device="cuda")
        out = torch.empty(m, nout, device="cuda")
        st = V(torch.cuda.current_stream().cuda_stream)
        call = lambda: f(V(g.data_ptr()), m, m, V(x.data_ptr()), nx, nx, U, V(part.data_ptr()), P,  # noqa: E731
                         V(out.data_ptr()), nout, nout, st)
        for _ in range(3):
            assert call() == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            call()
        e1.record()
        torch.cuda.synchronize()
        r[name] = e0.elapsed_time(e1) / 20
    res[f"mode{mode}"] = r
print(json.dumps(res, indent=1))
