"""Per-phase cycle breakdown of k_step_many (diagnostic build libfjsp_stamps.so, -DFJSP_STAMPS)."""
import ctypes, importlib, os, sys, json
os.environ["FJSP_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                      "multi-agent-rl-for-fjsp_amd", sys.argv[1] if len(sys.argv) > 1 else "libfjsp_stamps.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
ve = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
L = nat.lib()
L.fjsp_debug_stamps.argtypes = [ctypes.c_void_p]
names = ["synth_actions(+barrier)", "action_phase", "run_phase", "rewards|snapshot", "observe", "stores", "autoreset+next_obs", "-"]
if "fine" in (sys.argv[1] if len(sys.argv) > 1 else ""):
    names = ["synth_actions(+barrier)", "pickup", "agv", "machines", "packaging", "run_phase", "rewards+observe+stores|snapshot", "autoreset"]
for N in (4096,):
    for pipe, lds in ((1, 0), (1, 1), (0, 0)):   # pipelined: the sim wave's phases (emit wave not stamped)
        env = ve.FJSPVecEnv(N)
        nat.check(L.fjsp_set_option(env.handle, b"pipeline", pipe))
        nat.check(L.fjsp_set_option(env.handle, b"fused_lds", lds))
        env.reset(seeds=torch.arange(N))
        b = ve.Buffers(200, N, env.device, infos=False)
        env.rollout(200, buffers=b); torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 8)()
        L.fjsp_debug_stamps(buf)
        env.rollout(200, step0=200, buffers=b); torch.cuda.synchronize()
        L.fjsp_debug_stamps(buf)
        waves, steps = N // 64, 200
        tot = sum(buf[:8])
        print(json.dumps({"N": N, "pipeline": pipe, "lds": lds, "cycles_per_wave_step": tot / waves / steps,
                          "phases": {names[i]: round(buf[i] / waves / steps, 1) for i in range(8)}}))
