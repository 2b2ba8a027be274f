"""Bring-up aid: per-lane values k_step_ag records for workgroup 1 at step 0 (libfjsp_dbg.so)."""
import ctypes, os, sys
import numpy as np
os.environ["FJSP_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multi-agent-rl-for-fjsp_amd", "libfjsp_dbg.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests import gpu_util as G
L = G.native.lib()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
env = G.make_env(n)
G.native.check(L.fjsp_set_option(env.handle, b"agents", 1))
env.reset(seeds=torch.arange(n) * 3 + 1, num_orders=20)
env.rollout(1, action_seed=21, step0=0, policy="random")
torch.cuda.synchronize()
buf = np.zeros((8, 64), np.uint32)
L.fjsp_debug_dump(ctypes.c_void_p(buf.ctypes.data))
names = ["AM pend", "AM r1", "AM W6", "K pend", "K w0a", "K W23", "K W16", "K flag"]
for i in range(8):
    print(names[i], [hex(x) for x in buf[i][:40]])
