"""How often an agent's action is forced during an A2C collect (exactly one valid action in its
mask, so the sampled action does not depend on the actor's output): per agent, the share of
(step, env) samples and of 64-env tiles in which every env is forced.

usage: python scripts/diag_forced_actions.py [N] [batches]
"""
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
ve = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 3
env = ve.FJSPVecEnv(N)
L = A.VecMultiAgentA2C(env, seed=0)
L.reset(seeds=torch.arange(N), num_orders=25)
res = {a: {"forced": 0.0, "tiles_all_forced": 0.0} for a in A.AGENTS}
for b in range(nb):
    L.collect()
    m = L._bufs["masks"][:L.batch_size].int()                 # [T, 29, N]
    for i, a in enumerate(A.AGENTS):
        o, k = A.MASK_OFFS[i], A.N_ACTIONS[i]
        forced = m[:, o:o + k, :].sum(1) == 1                  # [T, N]
        res[a]["forced"] += float(forced.float().mean()) / nb
        tiles = forced.view(forced.shape[0], -1, 64).all(-1)
        res[a]["tiles_all_forced"] += float(tiles.float().mean()) / nb
    L.update()
print(json.dumps({"N": N, "batches": nb, "per_agent": {a: {k: round(v, 4) for k, v in r.items()} for a, r in res.items()}}))
