"""cProfile of the reference-API drop-in loop (bench.py dropin_latency's workload: FJSPParallelEnv
.step(dict) + a2c.py:298-305's agv reads, one env): where the host time of a step goes.
usage: python scripts/prof_dropin.py [steps]"""
import cProfile
import importlib
import io
import json
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

W = importlib.import_module("multi-agent-rl-for-fjsp_amd.FJSPParallelEnvWrapper")
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
env = W.FJSPParallelEnv()
env.reset(seed=0, options={"num_orders": 30})
rng = np.random.default_rng(0)
n_act = [env.action_space(a).n for a in env.possible_agents]
acts = [{a: int(rng.integers(0, n_act[i])) for i, a in enumerate(env.possible_agents)} for _ in range(steps)]
sim = env.unwrapped.simulation


def loop(n):
    for t in range(n):
        env.step(acts[t])
        _ = sim.agv.position
        _ = sim.agv.carrying_tray is not None
        if not env.agents:
            env.reset(options={"num_orders": 30})


loop(300)
t0 = time.perf_counter()
loop(steps)
plain = (time.perf_counter() - t0) / steps * 1e6
# the GPU part alone: launch + stream sync of the same kernel through ctypes, no Python around it
L, h = sim._L, sim._h
t0 = time.perf_counter()
for t in range(steps):
    L.fjsp_step(h, sim._act_ptr, None, 0, sim._packed.ref_full)
    L.fjsp_sync(h)
launch_sync = (time.perf_counter() - t0) / steps * 1e6
# the step server's request alone (doorbell + wait): the facade's inline mode (the action bytes
# in the doorbell's cache line), then with an actions buffer read by the kernel


def requests(inline):
    L.fjsp_server_start(h, None if inline else sim._act_ptr, 0, sim._packed.ref_full)
    req = (lambda: L.fjsp_server_step_actions(h, sim._act_ptr)) if inline else (lambda: L.fjsp_server_step(h))
    for t in range(100):
        assert req() == 0
    t0 = time.perf_counter()
    for t in range(steps):
        assert req() == 0
    us = (time.perf_counter() - t0) / steps * 1e6
    L.fjsp_server_stop(h)
    return us


server_buf = requests(False)
server_step = requests(True)   # the facade's own configuration again
env.reset(seed=1, options={"num_orders": 30})
pr = cProfile.Profile()
pr.enable()
loop(steps)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(json.dumps({"us_per_step": plain, "launch_plus_sync_us": launch_sync, "server_step_us": server_step,
                  "server_step_actions_buffer_us": server_buf}))
print(s.getvalue(), file=sys.stderr)
