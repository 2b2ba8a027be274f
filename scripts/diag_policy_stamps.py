"""Per-workgroup timeline of the fused policy kernel from a -DFJSP_STAMPS build
(libfjsp_pstamps.so, csrc/fjsp_policy.hip PST slots): on the observations of a real 4 096-env
collect, for each launch the span (s_memrealtime, 100 MHz), the workgroups per CU, and per role
the mean cycles of each phase (s_memtime) of the unforced workgroups.

usage: python scripts/diag_policy_stamps.py LIB [all|actors|values] [launches]
"""
import ctypes
import importlib
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")

LIB = sys.argv[1]
PART = sys.argv[2] if len(sys.argv) > 2 else "all"
LAUNCHES = int(sys.argv[3]) if len(sys.argv) > 3 else 32
N = 4096
P = ctypes.c_void_p
stream = torch.cuda.current_stream()
L = A.VecMultiAgentA2C(V.FJSPVecEnv(N), batch_size=256, seed=0)
L.reset(seeds=torch.arange(N), num_orders=25)
L.collect()
L.update()
L.roll_over()
L.collect()
torch.cuda.synchronize()
feats, masks = L._bufs["feats"], L._bufs["masks"]
lib = ctypes.CDLL(os.path.abspath(LIB))
f = lib.fjsp_a2c_policy
f.argtypes = [P, P, ctypes.c_int32, P, P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32, P, P, P, P]
lib.fjsp_debug_policy_stamps.argtypes = [P, ctypes.c_int32]
act = torch.zeros(8, N, dtype=torch.uint8, device="cuda")
val = torch.zeros(N, dtype=torch.float32, device="cuda")
buf = np.zeros((2048, 16), dtype=np.uint64)
# phases ending at stamp slots 2..9 (csrc/fjsp_policy.hip PST): actor forced check, inputs, layer 1 +
# h1 half 0, layer 2 half 0, layer 1 + h1 half 1, layer 2 half 1, logits, epilogue; critic -, inputs,
# layer 1, h1 hand-off, layer 2, h2 hand-off, layer 3 + value head, value sum
PH = ["s2", "s3", "s4", "s5", "s6", "s7", "s8", "s9"]
phase = defaultdict(lambda: np.zeros(len(PH)))
count = defaultdict(int)
forced_cyc = []
spans, per_cu_max, late_starts, clocks = [], [], [], []
for i in range(LAUNCHES + 4):
    t = 8 + i
    rc = f(P(feats[t].data_ptr()), P(masks[t].data_ptr()), N, P(L._pw_actor.data_ptr()), P(L._pw_critic.data_ptr()),
           P(L._rng.data_ptr()), 0, t, 0, None if PART == "values" else P(act.data_ptr()),
           None if PART == "actors" else P(val.data_ptr()), None, P(stream.cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    assert lib.fjsp_debug_policy_stamps(P(buf.ctypes.data), 1) == 0
    if i < 4:
        continue
    s = buf[buf[:, 0] != 0].astype(np.int64)
    t0 = s[:, 0].min()
    start, end = (s[:, 0] - t0) * 0.01, (s[:, 10] - t0) * 0.01   # us
    spans.append(float(end.max()))
    first_end = float(end.min())
    late_starts.append(int((start > first_end).sum()))
    cu = defaultdict(int)
    for r in s:
        hw, xcc = int(r[11]), int(r[12]) & 0xF
        cu[(xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF)] += 1
    per_cu_max.append(max(cu.values()))
    dur_rt = (s[:, 10] - s[:, 0]).astype(np.float64)
    ok = dur_rt > 50
    clocks.append(float(np.median((s[ok, 9] - s[ok, 1]) / dur_rt[ok] * 100.0)))   # MHz
    for r in s:
        role, forced = int(r[13]) & 0xFF, int(r[13]) >> 8
        if r[2] == 0:
            r[2] = r[1]
        if forced:
            forced_cyc.append(int(r[9] - r[1]))
            continue
        phase[role] += np.diff(r[1:10].astype(np.float64))
        count[role] += 1
out = {"lib": LIB, "part": PART, "launches": LAUNCHES, "span_us_median": float(np.median(spans)),
       "span_us_p10": float(np.percentile(spans, 10)), "span_us_p90": float(np.percentile(spans, 90)),
       "workgroups_started_after_first_exit_median": float(np.median(late_starts)),
       "max_workgroups_per_cu_median": float(np.median(per_cu_max)), "clock_mhz_median": float(np.median(clocks)),
       "forced_workgroup_cycles_mean": float(np.mean(forced_cyc)) if forced_cyc else None,
       "roles": {}}
names = ["pickup", "agv", "small", "big", "pkg_blue_1", "pkg_blue_2", "pkg_red", "pkg_green", "critic"]
for role in sorted(phase):
    c = count[role]
    out["roles"][names[role] if role < len(names) else str(role)] = {
        "unforced_per_launch": c / LAUNCHES,
        "cycles": {k: round(float(v / c)) for k, v in zip(PH, phase[role])},
        "total_cycles": round(float(phase[role].sum() / c))}
print(json.dumps(out, indent=1))
