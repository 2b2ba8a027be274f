"""The step server's traffic per env-step (for a PMC pass: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
around this script): N envs, K requests through fjsp_server_step with the actions rewritten in
pinned memory each step, the lean outputs (obs, masks, rewards, term, trunc, status) in HBM, then
one stop (the resident kernel leaves: one dispatch covering all K steps).  Prints JSON with the
wall time per request.  usage: python scripts/diag_server_pmc.py [N] [K]"""
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
env = V.FJSPVecEnv(N)
env.reset(seeds=torch.arange(N), num_orders=30)
rng = np.random.default_rng(0)
nact = np.array([3, 8, 3, 3, 3, 3, 3, 3]).reshape(8, 1)
acts = [((rng.integers(0, 256, (8, N)) * nact) >> 8).astype(np.uint8) for _ in range(64)]
hb = torch.zeros(8, N, dtype=torch.uint8).pin_memory()
hv = hb.numpy()
env.server_start(hb, autoreset=True, buffers=V.Buffers(1, N, env.device, infos=False))
t0 = time.perf_counter()
for t in range(K):
    hv[:] = acts[t & 63]
    env.server_step()
wall = (time.perf_counter() - t0) / K
env.server_stop()
torch.cuda.synchronize()
print(json.dumps({"envs": N, "requests": K, "us_per_request": wall * 1e6, "env_steps_per_s": N / wall,
                  "kernel": "k_step_server (one dispatch for all requests)"}))
