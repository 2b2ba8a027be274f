#!/usr/bin/env python3
"""The collect's fused launch (k_policy_step) split into its policy part and the env-step tail
of each 64-env tile, from a stamps build (scripts/build_diag.sh -> libfjsp_stamps.so, run with
FJSP_LIB pointing at it): per launch of one env group (launched alone and synchronised, so the
per-block stamp slots are not shared), for every tile's last actor workgroup the cycles from its
entry to the tail (slot 1 -> 14) and of the tail (14 -> 15), and the launch's HIP-event time.
Prints JSON.

usage: FJSP_LIB=.../libfjsp_stamps.so python scripts/diag_collect_tail.py [N] [steps] [warm_batches]"""
import ctypes
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")


def main(N=4096, steps=64, warm=1):
    L = A.VecMultiAgentA2C(V.FJSPVecEnv(N), batch_size=256, seed=0)
    L.reset(seeds=torch.arange(N), num_orders=25)
    for _ in range(warm):
        L.collect()
        L.update()
        L.roll_over()
    lib = A.nat.lib()
    lib.fjsp_debug_policy_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    buf = np.zeros(2048 * 16, dtype=np.uint64)
    lib.fjsp_debug_policy_stamps(buf.ctypes.data, 1)
    groups = L._collect_groups()
    st = torch.cuda.current_stream()
    pre, tail, ev_ms, phases, roles = [], [], [], [], []
    for t in range(steps):
        for e0, cnt in groups:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            L.policy_step(t, False, e0, cnt, st)
            b.record(st)
            torch.cuda.synchronize()
            ev_ms.append(a.elapsed_time(b))
            lib.fjsp_debug_policy_stamps(buf.ctypes.data, 1)
            s = buf.reshape(2048, 16).astype(np.int64)
            last = s[:, 15] > 0
            pre.append((s[last, 14] - s[last, 1]).tolist())
            roles.extend((s[last, 13] & 255).tolist())
            tail.append((s[last, 15] - s[last, 14]).tolist())
            # the tail's phases: 14 -> 2 actions + reward table, 2 -> 3 env_advance, 3 -> 4 rewards /
            # term / trunc / status, 4 -> 5 auto-reset, 5 -> 6 observation, 6 -> 15 state store
            cols = [14, 2, 3, 4, 5, 6, 15]
            phases.append(np.diff(s[last][:, cols], axis=1))
    P = np.array([x for l in pre for x in l])
    Tl = np.array([x for l in tail for x in l])
    per_launch_max_tail = [max(x) for x in tail if x]
    per_launch_max_end = [max(p + q for p, q in zip(x, y)) for x, y in zip(pre, tail) if x]
    res = {"envs": N, "groups": groups, "launches": len(ev_ms),
           "launch_ms_median": float(np.median(ev_ms)),
           "tail_cycles": {"mean": float(Tl.mean()), "p50": float(np.median(Tl)), "p90": float(np.percentile(Tl, 90)),
                           "max": float(Tl.max())},
           "entry_to_tail_cycles": {"mean": float(P.mean()), "p50": float(np.median(P)),
                                    "p90": float(np.percentile(P, 90)), "max": float(P.max())},
           "per_launch_max_tail_cycles_median": float(np.median(per_launch_max_tail)),
           "per_launch_max_entry_to_end_cycles_median": float(np.median(per_launch_max_end)),
           "tail_phase_cycles_mean": dict(zip(["actions_lut", "env_advance", "step_outputs", "autoreset", "observe",
                                               "state_store"], np.concatenate(phases).mean(0).tolist())),
           "last_role_share": {name: roles.count(r) / max(1, len(roles)) for r, name in enumerate(A.AGENTS)},
           "note": "cycles = s_memtime ticks (shader clock); the entry stamp is the tail workgroup's own"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:]))
