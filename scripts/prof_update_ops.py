"""torch.profiler view of the grouped A2C update (VecMultiAgentA2C.update) at N envs x 256
steps: device time per torch op (self), summed over 3 updates after 2 warm-up ones, top rows.

usage: python scripts/prof_update_ops.py [N] [rows]
"""
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
ROWS = int(sys.argv[2]) if len(sys.argv) > 2 else 45
L = A.VecMultiAgentA2C(V.FJSPVecEnv(N), batch_size=256, seed=0)
L.reset(seeds=torch.arange(N), num_orders=25)
for _ in range(2):
    L.collect()
    L.update()
    L.roll_over()
L.collect()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(3):
        L.update()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=ROWS, max_name_column_width=60))
