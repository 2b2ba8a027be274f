"""torch.profiler view of the grouped A2C update at N envs grouped by op and input shapes: where
the small copies / fills / reductions of the update's glue come from (device time, 3 updates).

usage: python scripts/prof_update_shapes.py [N] [rows]
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
ROWS = int(sys.argv[2]) if len(sys.argv) > 2 else 60
L = A.VecMultiAgentA2C(V.FJSPVecEnv(N), batch_size=256, seed=0)
L.reset(seeds=torch.arange(N), num_orders=25)
for _ in range(2):
    L.collect()
    L.update()
    L.roll_over()
L.collect()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    for _ in range(3):
        L.update()
    torch.cuda.synchronize()
ka = prof.key_averages(group_by_input_shape=True)
rows = [e for e in ka if e.key in ("aten::copy_", "aten::fill_", "aten::sum", "aten::cat", "aten::index", "aten::gather",
                                    "aten::mul", "aten::sub", "aten::add_", "aten::zeros", "aten::pow", "aten::to",
                                    "aten::index_put_", "aten::contiguous", "aten::clone")]
rows.sort(key=lambda e: -e.self_device_time_total)
for e in rows[:ROWS]:
    print(f"{e.key:22s} {e.count:5d} {e.self_device_time_total / 3 / 1e3:8.3f} ms/update  {str(e.input_shapes)[:150]}")
ks = prof.key_averages(group_by_stack_n=6)
rows = [e for e in ks if e.key == "aten::copy_"]
rows.sort(key=lambda e: -e.self_device_time_total)
print("--- copy_ by stack")
for e in rows[:15]:
    print(f"{e.count:5d} {e.self_device_time_total / 3 / 1e3:8.3f} ms/update")
    for fr in e.stack[:6]:
        print("      ", fr)
