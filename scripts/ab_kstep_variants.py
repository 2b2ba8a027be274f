"""A/B of the one-launch-per-step kernel variants of ONE library build (fjsp_step, canonical
order, actions in HBM): r05's k_step<canon> (option legacy_step), k_step_pf (read-ahead table
reads, direct stores) and k_step_pf<staged> (option step_staged).  N envs, interleaved rounds of
200 launches, HIP-event time per launch (median of rounds), outputs of every round byte-compared.

usage: python scripts/ab_kstep_variants.py [N] [rounds]"""
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 8
stream = torch.cuda.current_stream()
variants = {"legacy": {"legacy_step": 1}, "pf": {}, "pf_staged": {"step_staged": 1}}
envs = {}
for name, opts in variants.items():
    env = V.FJSPVecEnv(N)
    nat.check(nat.lib().fjsp_set_option(env.handle, b"timing", 0))
    for k, v in opts.items():
        nat.check(nat.lib().fjsp_set_option(env.handle, k.encode(), v))
    env.reset(seeds=torch.arange(N), num_orders=30)
    envs[name] = (env, V.Buffers(1, N, env.device, infos=False))
g = torch.Generator(device="cuda").manual_seed(5)
nact = torch.tensor([3, 8, 3, 3, 3, 3, 3, 3], dtype=torch.int32, device="cuda").view(8, 1)
acts = [((torch.randint(0, 256, (8, N), dtype=torch.int32, device="cuda", generator=g) * nact) >> 8).to(torch.uint8)
        for _ in range(200)]
ms = {k: [] for k in variants}
kern = {}
for r in range(ROUNDS + 1):
    outs = {}
    for name, (env, buf) in envs.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for a in acts:
            env.step(a, buffers=buf)
        e1.record(stream)
        torch.cuda.synchronize()
        if r:
            ms[name].append(e0.elapsed_time(e1) / len(acts))
        kern[name] = env.last_kernel()
        outs[name] = b"".join(getattr(buf, k).cpu().numpy().tobytes()
                              for k in ("obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "status"))
    ref = outs["legacy"]
    assert all(o == ref for o in outs.values()), "outputs differ"
print(json.dumps({"N": N, "rounds": ROUNDS, "launches_per_round": 200, "kernel": kern,
                  "us_per_launch_median": {k: float(np.median(v)) * 1e3 for k, v in ms.items()},
                  "us_per_launch_all": {k: [round(x * 1e3, 3) for x in v] for k, v in ms.items()},
                  "outputs_equal": True}))
