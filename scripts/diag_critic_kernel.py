#!/usr/bin/env python3
"""fjsp_a2c_critic_fused alone (the grouped update's one-pass critic), for counter passes and
A/B runs: U distinct synthetic states, `reps` launches per variant, HIP-event time per launch;
variants = values of an environment variable the library reads per call (FJSP_AB_VAR names it;
none by default), alternated per launch, outputs compared bitwise with the first variant's.
Prints JSON.  (r05: FJSP_CRITIC_RING=1/2/3, the weight ring depth of a since-removed variant
build: profiles/r05/critic_ring_depth_ab.json.)

usage: python scripts/diag_critic_kernel.py [U] [reps] [value value ..]"""
import ctypes
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")


def main(U=540000, reps=10, rings="1"):
    torch.manual_seed(0)
    _, critic = A.init_networks(seed=3, device="cuda")
    xT = (torch.rand(38, U, device="cuda") * torch.randint(0, 30, (38, 1), device="cuda")).float()
    x = torch.nn.functional.pad(xT.t(), (0, 2)).contiguous()
    nu = torch.randint(1, 6, (U,), device="cuda").double()
    sr = torch.randn(U, device="cuda", dtype=torch.float64) * nu * 8 * 3
    coef = A.critic_coef_sums(nu, sr, sr * sr / (8 * nu) + 1.0, float(nu.sum())).contiguous()
    ps = [p.detach() for p in critic.parameters()]
    cw = A.pack_critic_weights(*ps)
    w3t, w2t = A.pack_mfma(ps[4].t()).reshape(-1), A.pack_mfma(ps[2].t()).reshape(-1)
    E = lambda *sh: torch.empty(*sh, dtype=torch.float32, device="cuda")  # noqa: E731
    h1, h2, g2, g1, g3 = E(U, 256), E(U, 256), E(U, 256), E(U, 256), E(U, 128)
    tiles = -(-U // 32)
    part = E(tiles, A.nat.CRITIC_FUSED_PW)
    loss = torch.empty(tiles, dtype=torch.float64, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = torch.cuda.current_stream()
    variants = rings.split(",")
    ms = {v: [] for v in variants}
    ref, same = None, {}
    for _ in range(reps):
        for v in variants:
            if os.environ.get("FJSP_AB_VAR"):
                os.environ[os.environ["FJSP_AB_VAR"]] = v
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            A.nat.check(A.nat.lib().fjsp_a2c_critic_fused(P(x), U, P(cw), P(w3t), P(w2t), P(coef), P(h1), P(h2), P(g3),
                                                          P(g2), P(g1), P(part), P(loss), None,
                                                          ctypes.c_void_p(st.cuda_stream)))
            e1.record()
            torch.cuda.synchronize()
            ms[v].append(e0.elapsed_time(e1))
            out = [t.clone() for t in (h1, h2, g3, g2, g1, part, loss)]
            if ref is None:
                ref = out
            same[v] = same.get(v, True) and all(torch.equal(a.view(torch.uint8), b.view(torch.uint8))
                                                 for a, b in zip(ref, out))
    mfmas = tiles * 2448
    med = {v: sorted(t[2:])[len(t[2:]) // 2] for v, t in ms.items()}
    print(json.dumps({"U": U, "ms": ms, "ms_median": med, "bit_equal_to_first": same, "mfma_per_launch": mfmas,
                      "mfma_util_at_2.4GHz": {v: mfmas * 32 / (1024 * 2.4e9 * m * 1e-3) for v, m in med.items()},
                      "hbm_bytes_written_per_launch": U * (4 * 256 * 4 + 128 * 4)}), flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(*([int(x) for x in a[:2]] + ([",".join(a[2:])] if len(a) > 2 else [])))
