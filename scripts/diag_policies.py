"""Diagnostic: fused-rollout cost per step vs policy and num_orders (episode ends desync the
lanes of a wave, so every lane's reset is paid by the whole wave)."""
import importlib, json, os, sys
if len(sys.argv) > 1:   # diagnostic library variant, e.g. libfjsp_rinl.so
    os.environ["FJSP_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                          "multi-agent-rl-for-fjsp_amd", sys.argv[1])
NS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [4096, 65536]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
ve = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
for N in NS:
    for policy in ("random", "masked", "heuristic"):
        for no in (30, 5, 2):
            env = ve.FJSPVecEnv(N)
            env.reset(seeds=torch.arange(N), num_orders=no)
            K = 200
            b = ve.Buffers(K, N, env.device, infos=False)
            env.rollout(K, policy=policy, buffers=b)
            ms, ends = [], 0
            for r in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                env.rollout(K, step0=(r + 1) * K, policy=policy, buffers=b)
                e1.record(); torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
                ends += int((b.term | b.trunc).sum())
            print(json.dumps({"lib": os.path.basename(os.environ.get("FJSP_LIB", "libfjsp.so")), "N": N, "policy": policy, "num_orders": no, "kernel": env.last_kernel(),
                              "us_per_step": round(sum(ms) / len(ms) / K * 1e3, 3),
                              "episode_ends_per_1k_env_steps": round(ends / (5 * K * N) * 1e3, 2)}), flush=True)
            del env, b
