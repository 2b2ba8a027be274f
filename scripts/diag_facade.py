"""Per-step latency of the reference-API drop-in (N = 1, dict in / dict out) vs the reference's
~115 us/step."""
import importlib, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
W = importlib.import_module("multi-agent-rl-for-fjsp_amd.FJSPParallelEnvWrapper")
env = W.FJSPParallelEnv()
obs, _ = env.reset(seed=0, options={"num_orders": 30})
rng = np.random.default_rng(0)
n_act = {a: env.action_space(a).n for a in env.possible_agents}
acts = [{a: int(rng.integers(0, n_act[a])) for a in env.possible_agents} for _ in range(2000)]
for t in range(100):
    obs, r, te, tr, info = env.step(acts[t])
    if not env.agents:
        env.reset(options={"num_orders": 30})
t0 = time.perf_counter()
for t in range(2000):
    obs, r, te, tr, info = env.step(acts[t])
    if not env.agents:
        env.reset(options={"num_orders": 30})
dt = (time.perf_counter() - t0) / 2000
print(json.dumps({"facade_step_us": dt * 1e6, "steps": 2000}))
