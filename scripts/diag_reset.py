"""Diagnostic: fjsp_reset cost vs num_orders (seeded and continued streams)."""
import importlib, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
ve = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
N = 4096
env = ve.FJSPVecEnv(N)
b = ve.Buffers(1, N, env.device, infos=False)
for seeded in (True, False):
    for no in (0, 1, 5, 10, 30, 60):
        ms = []
        for r in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            env.reset(seeds=torch.arange(N) if seeded else None, num_orders=no, buffers=b)
            e1.record(); torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        print(json.dumps({"seeded": seeded, "num_orders": no, "us": [round(m * 1e3, 1) for m in ms]}), flush=True)
