"""Per-phase cycle breakdown of the one-launch-per-step kernel k_step<canon> (fjsp_step, actions
from HBM) at N envs, from the stamps build (scripts/build_diag.sh -> libfjsp_stamps.so).

Slots (k_step / step_and_emit): 0 entry -> reward table in LDS -> state + action loads landed,
1 action phase, 2 run phase, 3 rewards, 4 observe, 5 term / trunc / status, 6 auto-reset,
7 state store drained.  Lane 0 of every wave adds its cycles; printed per wave-launch.

usage: python scripts/diag_kstep_stamps.py [N] [launches]"""
import ctypes
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FJSP_LIB", os.path.join(REPO, "multi-agent-rl-for-fjsp_amd", "libfjsp_stamps.so"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
L = nat.lib()
L.fjsp_debug_stamps.argtypes = [ctypes.c_void_p]
env = V.FJSPVecEnv(N)
env.reset(seeds=torch.arange(N))
g = torch.Generator(device="cuda").manual_seed(3)
nact = torch.tensor([3, 8, 3, 3, 3, 3, 3, 3], dtype=torch.int32, device="cuda").view(1, 8, 1)
acts = ((torch.randint(0, 256, (K, 8, N), dtype=torch.int32, device="cuda", generator=g) * nact) >> 8).to(torch.uint8)
b = V.Buffers(1, N, env.device, infos=False)
for t in range(20):
    env.step(acts[t], buffers=b)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 8)()
L.fjsp_debug_stamps(buf)   # clears
for t in range(K):
    env.step(acts[t], buffers=b)
torch.cuda.synchronize()
L.fjsp_debug_stamps(buf)
names = ["entry_lut_state_loads", "action_phase", "run_phase", "rewards", "observe", "term_trunc_status",
         "autoreset", "state_store_drain"]
waves = (N + 63) // 64
per = {names[i]: round(buf[i] / waves / K, 1) for i in range(8)}
print(json.dumps({"N": N, "launches": K, "kernel": env.last_kernel(), "cycles_per_wave_launch": per,
                  "total": round(sum(buf) / waves / K, 1)}))
