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
L.fjsp_debug_pgstamps.argtypes = [ctypes.c_void_p]
names = ["synth_actions(+barrier)", "action_phase", "run_phase", "rewards|snapshot", "observe", "stores", "autoreset+next_obs", "-"]
if "fine" in (sys.argv[1] if len(sys.argv) > 1 else ""):
    names = ["synth_actions(+barrier)", "pickup", "agv", "machines", "packaging", "run_phase", "rewards+observe+stores|snapshot", "autoreset"]
for N in (4096,):
    cfgs = ((1, 1, 1), (1, 1, 0), (1, 0, 0), (0, 0, 0))
    for pipe, lds, pg in cfgs[:int(os.environ.get("STAMP_CFGS", "4"))]:   # pipelined: the sim wave's phases
        env = ve.FJSPVecEnv(N)
        nat.check(L.fjsp_set_option(env.handle, b"pipeline", pipe))
        nat.check(L.fjsp_set_option(env.handle, b"fused_lds", lds))
        nat.check(L.fjsp_set_option(env.handle, b"predraw", pg))
        env.reset(seeds=torch.arange(N))
        b = ve.Buffers(200, N, env.device, infos=False)
        env.rollout(200, buffers=b); torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 8)()
        L.fjsp_debug_stamps(buf)
        pgb = (ctypes.c_ulonglong * 8)()
        L.fjsp_debug_pgstamps(pgb)
        env.rollout(200, step0=200, buffers=b); torch.cuda.synchronize()
        L.fjsp_debug_stamps(buf)
        L.fjsp_debug_pgstamps(pgb)
        waves, steps = N // 64, 200
        tot = sum(buf[:8])
        print(json.dumps({"N": N, "pipeline": pipe, "lds": lds, "predraw": pg, "kernel": env.last_kernel(), "cycles_per_wave_step": tot / waves / steps,
                          "phases": {names[i]: round(buf[i] / waves / steps, 1) for i in range(8)},
                          "predraw_wave": {"busy_cycles_per_step": pgb[0] / max(1, pgb[3]),
                                           "active_step_frac": pgb[1] / max(1, pgb[3]),
                                           "busy_cycles_per_active_step": pgb[2] / max(1, pgb[1])},
                          "emit_waves_busy_cycles_per_step": [pgb[4] / max(1, pgb[5]), pgb[6] / max(1, pgb[7])]}))
