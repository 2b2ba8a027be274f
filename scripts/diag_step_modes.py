"""Diagnostic: us per step of the one-launch-per-step kernel (k_step, actions from HBM) against
the fused k_step_many with global or LDS tables, at N envs (4096 by default)."""
import importlib, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
ve = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
env = ve.FJSPVecEnv(N)
env.reset(seeds=torch.arange(N))
K = 200
acts = torch.randint(0, 256, (K, 8, N), dtype=torch.int32, device=env.device)
nact = torch.tensor([3, 8, 3, 3, 3, 3, 3, 3], dtype=torch.int32, device=env.device).view(1, 8, 1)
acts = ((acts * nact) >> 8).to(torch.uint8).contiguous()
sb = ve.Buffers(1, N, env.device, infos=False)
for t in range(20):
    env.step(acts[t], buffers=sb)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for t in range(K):
    env.step(acts[t], buffers=sb)
e1.record(); torch.cuda.synchronize()
print(json.dumps({"mode": "k_step (launch per step)", "kernel": env.last_kernel(), "us_per_step": e0.elapsed_time(e1) * 1e3 / K}))
for lds in (0, 1):
    nat.check(nat.lib().fjsp_set_option(env.handle, b"fused_lds", lds))
    b = ve.Buffers(K, N, env.device, infos=True)
    env.rollout(K, buffers=b, infos=True); torch.cuda.synchronize()
    e0.record(); env.rollout(K, step0=K, buffers=b, infos=True); e1.record(); torch.cuda.synchronize()
    print(json.dumps({"mode": "fused, full outputs", "kernel": env.last_kernel(), "us_per_step": e0.elapsed_time(e1) * 1e3 / K}))
