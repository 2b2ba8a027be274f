"""Diagnostic: us per step of the default fused kernel at N envs for the library FJSP_LIB
(timing builds with parts switched off; not part of the bench contract)."""
import importlib, json, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
ve = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
K = int(os.environ.get("K", "200"))
for N in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4096").split(",")]:
    env = ve.FJSPVecEnv(N, **({"max_episode_steps": int(os.environ["MAX_STEPS"])} if os.environ.get("MAX_STEPS") else {}))
    env.reset(seeds=torch.arange(N))
    b = ve.Buffers(K, N, env.device, infos=False)
    for f in [x for x in os.environ.get("NULL_OUTS", "").split(",") if x]:   # outputs not written
        setattr(b, f, None)
    env.rollout(K, buffers=b); torch.cuda.synchronize()
    ms = []
    for r in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); env.rollout(K, step0=(r + 1) * K, buffers=b); e1.record(); torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    print(json.dumps({"lib": os.path.basename(os.environ.get("FJSP_LIB", "libfjsp.so")), "N": N, "kernel": env.last_kernel(),
                      "null": os.environ.get("NULL_OUTS", ""), "us_per_step": min(ms) * 1e3 / K, "us_med": sorted(ms)[2] * 1e3 / K}), flush=True)
