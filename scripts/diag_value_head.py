"""The critic's value head (128 -> 1) over B rows: forward and weight-gradient variants (GEMM
with N = 1, split-K batched GEMM, mv), HIP-event us, median of 20.

usage: python scripts/diag_value_head.py [B]
"""
import json
import sys

import numpy as np
import torch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 540097
x = torch.randn(B, 128, device="cuda")
W = torch.randn(1, 128, device="cuda")
b = torch.randn(1, device="cuda")
gy = torch.randn(B, 1, device="cuda")


def timed(fn, reps=20):
    v = []
    for r in range(reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if r >= 3:
            v.append(e0.elapsed_time(e1) * 1e3)
    return round(float(np.median(v)), 1)


c = max(1, min(64, B // 8192))
bc = B // c
res = {"B": B,
       "fwd_addmm": timed(lambda: torch.addmm(b, x, W.t())),
       "fwd_mv": timed(lambda: torch.mv(x, W[0]) + b),
       "gW_splitk_bmm": timed(lambda: torch.bmm(gy[:c * bc].reshape(c, bc, 1).transpose(1, 2),
                                                x[:c * bc].reshape(c, bc, 128)).sum(0)),
       "gW_mm": timed(lambda: gy.t() @ x),
       "gW_mv": timed(lambda: torch.mv(x.t(), gy[:, 0])),
       "gx_outer": timed(lambda: gy * W)}
print(json.dumps(res))
