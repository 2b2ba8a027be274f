"""Which torch ops the grouped A2C update launches (VecMultiAgentA2C.update at N envs x 256
steps): per (op, input shapes) the calls per update and device time, sorted by calls — the small
launches that make up the update's glue.  usage: python scripts/prof_update_calls.py [N] [rows]"""
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
ROWS = int(sys.argv[2]) if len(sys.argv) > 2 else 70
L = A.VecMultiAgentA2C(V.FJSPVecEnv(N), batch_size=256, seed=0)
L.reset(seeds=torch.arange(N), num_orders=25)
for _ in range(2):
    L.collect()
    L.update()
    L.roll_over()
L.collect()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    L.update()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="count", row_limit=ROWS, max_name_column_width=40,
                                                         max_shapes_column_width=70))
print(prof.key_averages(group_by_stack_n=4).table(sort_by="count", row_limit=40, max_name_column_width=40))
