"""The grouped update's critic pass alone (forward + backward of the 38-256-256-128-1 MLP over
the batch's distinct global states, B rows) in variants: nn.Linear autograd, the split-K
weight gradient with padding copies (_LinearSplitK before), split-K over views, and rows
rounded up to a multiple of 256.  HIP-event ms, median of 10.

usage: python scripts/diag_critic_gemm.py [B] [mode,mode..]
"""
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 540097
dev = torch.device("cuda")
torch.manual_seed(0)
critic = A.CriticNet(A.GLOBAL_DIM).to(dev)
gt = torch.randn(A.GLOBAL_DIM, B + 256, device=dev)


class PadSplitK(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        return torch.addmm(b, x, W.t())

    @staticmethod
    def backward(ctx, gy):
        x, W = ctx.saved_tensors
        n = x.shape[0]
        c = max(1, min(64, n // 8192))
        bc = -(-n // c)
        pad = c * bc - n
        xp = torch.nn.functional.pad(x, (0, 0, 0, pad)).view(c, bc, -1)
        gp = torch.nn.functional.pad(gy, (0, 0, 0, pad)).view(c, bc, -1)
        return gy @ W, torch.bmm(gp.transpose(1, 2), xp).sum(0), gy.sum(0)


def fwd(x, mode):
    if mode == "fused":
        return A.mlp_forward(critic.net, x)
    for m in critic.net:
        if isinstance(m, torch.nn.Linear):
            if mode == "linear":
                x = m(x)
            elif mode == "padsplitk":
                x = PadSplitK.apply(x, m.weight, m.bias)
            else:
                x = A._LinearSplitK.apply(x, m.weight, m.bias, False)
        else:
            x = m(x)
    return x


def timed(fn, reps=10):
    v = []
    for r in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            v.append(e0.elapsed_time(e1))
    return round(float(np.median(v)), 3)


res = {"B": B}
modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["linear", "padsplitk", "splitk", "fused"]
for mode in modes:
    for rows in (B, -(-B // 256) * 256)[:1 if len(sys.argv) > 2 else 2]:
        x = gt[:, :rows].t()

        def f_only():
            with torch.no_grad():
                fwd(x, mode)

        def fb():
            critic.zero_grad(set_to_none=True)
            fwd(x, mode).sum().backward()
        res[f"{mode}_{rows}"] = {"fwd_ms": timed(f_only), "fwd_bwd_ms": timed(fb)}
        print(json.dumps({f"{mode}_{rows}": res[f"{mode}_{rows}"]}), flush=True)
flop = 2 * B * sum(m.weight.numel() for m in critic.net if isinstance(m, torch.nn.Linear))
res["fwd_gflop"] = flop / 1e9
print(json.dumps(res))
