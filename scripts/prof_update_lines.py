#!/usr/bin/env python3
"""Which Python lines of the grouped A2C update launch its small kernels: one update at N envs x
256 steps under torch.profiler with stacks, the torch ops grouped by their 4 innermost frames,
sorted by device time.  usage: python scripts/prof_update_lines.py [N] [rows]"""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ROWS = int(sys.argv[2]) if len(sys.argv) > 2 else 60
L = A.VecMultiAgentA2C(V.FJSPVecEnv(N), batch_size=256, seed=0)
L.reset(seeds=torch.arange(N), num_orders=25)
for _ in range(4):
    L.collect()
    L.update()
    L.roll_over()
L.collect()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    L.update()
    torch.cuda.synchronize()
ev = [e for e in prof.key_averages(group_by_stack_n=4) if e.device_time_total > 0 and e.stack]
ev.sort(key=lambda e: -e.self_device_time_total)
tot = sum(e.self_device_time_total for e in ev)
print(f"device time of ops with a Python stack: {tot / 1e3:.3f} ms")
for e in ev[:ROWS]:
    frames = [f for f in e.stack if "a2c_vec" in f or "shard_learner" in f or "distributed" in f][:3]
    print(f"{e.self_device_time_total / 1e3:8.3f} ms {e.count:4d}x  {e.key[:38]:38s} {' <- '.join(frames)}")
