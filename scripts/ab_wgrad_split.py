"""A/B of the critic's split-K weight-gradient GEMMs (a2c_vec._splitk_wgrad: gy^T x over U distinct
states as c batched chunks, summed) for the chunk count c, at the update's shapes (U = 698 284
distinct global states of a 4 096 x 256 batch, layers 256x256, 128x256, 256x40).  Median ms of
10 calls per (layer, c); max relative difference to c = 64 (the r05 choice).
usage: python scripts/ab_wgrad_split.py [U]"""
import json
import sys

import torch

U = int(sys.argv[1]) if len(sys.argv) > 1 else 698284
torch.manual_seed(0)
layers = {"W2": (256, 256), "W3": (128, 256), "W1": (256, 40)}
h1 = torch.randn(U, 256, device="cuda")
res = {}


def wgrad(gy, x, c):
    B = x.shape[0]
    bc = B // c
    xc = x[:c * bc].reshape(c, bc, -1)
    gc = gy[:c * bc].reshape(c, bc, -1)
    gW = torch.bmm(gc.transpose(1, 2), xc).sum(0)
    if c * bc < B:
        gW += gy[c * bc:].t() @ x[c * bc:]
    return gW


for name, (o, i) in layers.items():
    gy = torch.randn(U, o, device="cuda")
    x = torch.randn(U, 40, device="cuda")[:, :i] if i == 40 else torch.randn(U, i, device="cuda")
    ref = wgrad(gy, x, 64)
    out = {}
    for c in (16, 32, 64, 128, 256, 512):
        for _ in range(2):
            wgrad(gy, x, c)
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g = wgrad(gy, x, c)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        out[c] = {"ms": ts[len(ts) // 2], "max_rel_diff_vs_c64": float(((g - ref).abs().max() / ref.abs().max()))}
    res[name] = out
print(json.dumps({"U": U, "layers": res}))
