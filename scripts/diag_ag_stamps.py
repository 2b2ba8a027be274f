"""Per-wave cycles per epoch of k_step_ag (diagnostic build libfjsp_stamps.so)."""
import ctypes, os, sys, json
os.environ["FJSP_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                      "multi-agent-rl-for-fjsp_amd", sys.argv[1] if len(sys.argv) > 1 else "libfjsp_stamps.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests import gpu_util as G
L = G.native.lib()
L.fjsp_debug_agstamps.argtypes = [ctypes.c_void_p]
L.fjsp_debug_pgstamps.argtypes = [ctypes.c_void_p]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
env = G.make_env(N)
env.reset(seeds=torch.arange(N))
b = G.vec_env.Buffers(200, N, env.device, infos=False)
env.rollout(200, buffers=b); torch.cuda.synchronize()
ag = (ctypes.c_ulonglong * 64)(); pg = (ctypes.c_ulonglong * 8)()
L.fjsp_debug_agstamps(ag); L.fjsp_debug_pgstamps(pg)
env.rollout(200, step0=200, buffers=b); torch.cuda.synchronize()
L.fjsp_debug_agstamps(ag); L.fjsp_debug_pgstamps(pg)
ep = max(1, ag[16])
names = ["AM", "E0", "K", "E1", "P", "PD", "E2", "E3"]
print(json.dumps({"N": N, "kernel": env.last_kernel(), "per_epoch": {names[w]: {"busy": round(ag[2 * w] / ep), "wait_or_post": round(ag[2 * w + 1] / ep)} for w in range(8) if names[w] != "PD"},
                  "AM_t": {"top": round(ag[18] / ep), "after_reset_check": round(ag[19] / ep), "after_apply": round(ag[20] / ep), "after_mexec": round(ag[21] / ep), "after_post": round(ag[22] / ep), "after_mrun": round(ag[23] / ep)},
                  "P_t": {"after_synth": round(ag[33] / ep), "after_fresh_wait": round(ag[34] / ep), "after_pickup": round(ag[35] / ep), "after_flag": round(ag[36] / ep), "after_agv": round(ag[37] / ep), "after_writes": round(ag[38] / ep)}, "E3_t": {m: round(ag[40 + i] / ep) for i, m in enumerate(["after_pickup_post", "after_snapshot", "after_stores", "after_fresh_wait", "after_pickup_exec"])},
                  "E2_t": {m: round(ag[46 + i] / ep) for i, m in enumerate(["top", "after_snapshot", "after_stores"])}, "wall_cycles_per_epoch": round(ag[24] / ep), "last_arrival_frac": {names[w]: round(ag[25 + w] / ep, 3) for w in range(8) if names[w] != "PD"}, "simd_of_role": {names[w]: (ag[17] >> (4 * w)) & 3 for w in range(8)},
                  "predraw": {"busy_per_step": pg[0] / max(1, pg[3]), "active_frac": pg[1] / max(1, pg[3]), "busy_active": pg[2] / max(1, pg[1]), "to_draw_active": ag[52] / max(1, pg[1]), "draw_active": ag[53] / max(1, pg[1])}}))
