"""Per-launch fixed cost of k_step_ag and the phase breakdown of k_step (one launch per step).

usage: python scripts/diag_fixed_cost.py [sweep|stamps] [N]
  sweep   product library: HIP-event time of k_step_ag launches of K = 1 .. 1024 steps -> the
          per-step slope and the per-launch intercept (least squares)
  stamps  diagnostic build libfjsp_stamps.so (-DFJSP_STAMPS): k_step_ag's prologue (tables into
          LDS), copy-out and whole-launch cycles per workgroup, and k_step's cycles per phase
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
mode = sys.argv[1] if len(sys.argv) > 1 else "sweep"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
if mode == "stamps":
    os.environ["FJSP_LIB"] = os.path.join(REPO, "multi-agent-rl-for-fjsp_amd", "libfjsp_stamps.so")
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from tests import gpu_util as G  # noqa: E402

L = G.native.lib()
env = G.make_env(N)
env.reset(seeds=torch.arange(N))
stream = torch.cuda.current_stream()
if mode == "sweep":
    b = G.vec_env.Buffers(1024, N, env.device, infos=False)
    env.rollout(1024, buffers=b)
    torch.cuda.synchronize()
    res, t = {}, 1024
    for K in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024):
        ms = []
        for r in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            env.rollout(K, step0=t, buffers=b)
            e1.record(stream)
            torch.cuda.synchronize()
            t += K
            if r:
                ms.append(e0.elapsed_time(e1))
        res[K] = float(np.median(ms))
    Ks = np.array(list(res), float)
    y = np.array([res[k] for k in res]) * 1e3
    A = np.stack([Ks, np.ones_like(Ks)], 1)
    slope, icpt = np.linalg.lstsq(A, y, rcond=None)[0]
    print(json.dumps({"N": N, "kernel": env.last_kernel(), "us_per_launch": {int(k): round(v * 1e3, 2) for k, v in res.items()},
                      "fit_us_per_step": round(float(slope), 4), "fit_intercept_us": round(float(icpt), 2)}))
else:
    L.fjsp_debug_agstamps.argtypes = [ctypes.c_void_p]
    L.fjsp_debug_stamps.argtypes = [ctypes.c_void_p]
    wgs = (N + 63) // 64
    out = {"N": N}
    for K in (20, 1024):
        b = G.vec_env.Buffers(K, N, env.device, infos=False)
        env.rollout(K, buffers=b)
        torch.cuda.synchronize()
        ag = (ctypes.c_ulonglong * 64)()
        L.fjsp_debug_agstamps(ag)   # reads and clears
        for r in range(3):
            env.rollout(K, step0=(r + 1) * K, buffers=b)
        torch.cuda.synchronize()
        L.fjsp_debug_agstamps(ag)
        per = 3 * wgs
        out[f"k_step_ag_K{K}"] = {"prologue_cycles": ag[56] / per, "copy_out_cycles": ag[57] / per,
                                  "launch_cycles": ag[58] / per, "loop_cycles": ag[24] / per}
    sb = G.vec_env.Buffers(1, N, env.device, infos=False)
    acts = (torch.randint(0, 1 << 16, (300, 8, N), device="cuda") %
            torch.tensor([3, 8, 3, 3, 3, 3, 3, 3], device="cuda").view(1, 8, 1)).to(torch.uint8)
    for t in range(50):
        env.step(acts[t], buffers=sb)
    torch.cuda.synchronize()
    st = (ctypes.c_ulonglong * 8)()
    L.fjsp_debug_stamps(st)
    for t in range(50, 250):
        env.step(acts[t], buffers=sb)
    torch.cuda.synchronize()
    L.fjsp_debug_stamps(st)
    names = ["entry+LUT+state loads", "action phase", "run phase", "rewards", "observe", "term/trunc/status",
             "autoreset+next obs", "state store drained"]
    per = 200 * wgs
    out["k_step_cycles_per_wave_step"] = {names[i]: round(st[i] / per) for i in range(8)}
    out["k_step_total"] = round(sum(st) / per)
    print(json.dumps(out))
