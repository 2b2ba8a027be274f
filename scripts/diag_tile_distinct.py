#!/usr/bin/env python3
"""Distinct actor inputs per 64-env tile of the collect (diagnostic for an in-tile dedup of the
policy's MLPs): over one 256 x N batch after `warm` training batches, per agent, the share of
(step, tile) pairs whose 64 inputs hold <= 32 distinct rows (then one 32-env column tile would
do the MLP), the mean distinct count, and the share of tiles that are fully forced (one valid
action in every env: no MLP at all).  Prints JSON.

usage: python scripts/diag_tile_distinct.py [N] [warm] [trained]"""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")


def main(N=4096, warm=1, trained=0):
    L = A.VecMultiAgentA2C(V.FJSPVecEnv(N), batch_size=256, seed=0)
    if trained:
        L.load_state_dicts(A.load_npz_weights(os.path.join(REPO, "tests", "golden", "trained_policy.npz")))
    L.reset(seeds=torch.arange(N), num_orders=25)
    for _ in range(warm):
        L.collect()
        L.update()
        L.roll_over()
    L.collect()
    torch.cuda.synchronize()
    b = L._bufs
    T = L.batch_size
    feats, masks = b["feats"][:T], b["masks"][:T]                    # [T, 38, N], [T, 29, N]
    x = A.actor_inputs(feats, L.gidx).view(A.NA, A.DPAD, T, N // 64, 64)   # [8, 13, T, tiles, 64]
    # a row hash per (agent, t, tile, env): the 13 words' bits mixed
    bits = x.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    h = torch.zeros(A.NA, T, N // 64, 64, dtype=torch.int64, device=x.device)
    for c in range(A.DPAD):
        h = A._fmix64(h * 0x100000001B3 + bits[:, c] + c + 1)
    hs = torch.sort(h, dim=-1).values
    distinct = 1 + (hs[..., 1:] != hs[..., :-1]).sum(-1)                   # [8, T, tiles]
    nvalid = torch.stack([masks[:, o:o + k].to(torch.int32).sum(1) for o, k in zip(A.MASK_OFFS, A.N_ACTIONS)])
    forced = (nvalid.view(A.NA, T, N // 64, 64) == 1).all(-1)               # [8, T, tiles]
    res = {"envs": N, "warm_batches": warm, "trained": bool(trained), "per_agent": {}}
    for a, name in enumerate(A.AGENTS):
        d = distinct[a].float()
        mlp = ~forced[a]
        res["per_agent"][name] = {
            "forced_tile_share": float(forced[a].float().mean()),
            "mean_distinct_per_tile": float(d.mean()),
            "share_le32_of_mlp_tiles": float((d[mlp] <= 32).float().mean()) if bool(mlp.any()) else None,
            "share_le16_of_mlp_tiles": float((d[mlp] <= 16).float().mean()) if bool(mlp.any()) else None}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:]))
