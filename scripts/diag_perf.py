"""Diagnostic timing of the fused step kernel variants (not part of the bench contract)."""
import importlib, json, sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
ve = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
res = []
K = 200
for N in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4096,16384,65536").split(",")]:
    env = ve.FJSPVecEnv(N)
    env.reset(seeds=torch.arange(N))
    full = ve.Buffers(K, N, env.device, infos=False)
    none = ve.Buffers(1, N, env.device, infos=False)
    for k in ["obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "status"]:
        setattr(none, k, None)
    for lds in (0, 1):
        nat.check(nat.lib().fjsp_set_option(env.handle, b"fused_lds", lds))
        for name, b in (("all", full), ("none", none)):
            env.rollout(K, buffers=b); torch.cuda.synchronize()
            ms = []
            for r in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(); env.rollout(K, step0=(r + 1) * K, buffers=b); e1.record(); torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            m = min(ms)
            d = {"N": N, "lds": lds, "outputs": name, "ms_per_launch": m, "us_per_step": m * 1e3 / K,
                 "env_steps_per_s": N * K / (m * 1e-3)}
            print(json.dumps(d), flush=True)
            res.append(d)
    del env
