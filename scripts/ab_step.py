"""A/B timing of the bench kernel (k_step_ag at N envs, 1024-step launches, uniform-random
actions): variants = (library, option, value) run interleaved, HIP-event time per launch,
median and mean per variant, plus a byte comparison of each variant's first launch with the
first variant's.  Libraries are driven through raw ctypes (fjsp_create / reset / step_many /
set_option have kept their signatures since ABI 3), so an older build can be timed beside the
current one.

usage: python scripts/ab_step.py [N] [reps] [lib[:option=value]] ...
  e.g. ab_step.py 4096 8 multi-agent-rl-for-fjsp_amd/libfjsp.so:xcd_map=0 multi-agent-rl-for-fjsp_amd/libfjsp.so:xcd_map=1
  (option nostatus=1: the launch without the status output)
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import importlib  # noqa: E402

nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 8
specs = sys.argv[3:] or [nat.LIB_PATH + ":xcd_map=0", nat.LIB_PATH + ":xcd_map=1"]
K = 1024
stream = torch.cuda.current_stream()
P = ctypes.c_void_p


def open_lib(path):
    L = ctypes.CDLL(os.path.abspath(path))
    L.fjsp_create.argtypes = [ctypes.POINTER(nat.fjsp_config), ctypes.c_int32, ctypes.c_int32, P, ctypes.POINTER(P)]
    L.fjsp_reset.argtypes = [P, P, P, ctypes.c_int32, ctypes.POINTER(nat.fjsp_out)]
    L.fjsp_step_many.argtypes = [P, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32,
                                 ctypes.c_int32, ctypes.POINTER(nat.fjsp_out)]
    L.fjsp_set_option.argtypes = [P, ctypes.c_char_p, ctypes.c_int64]
    L.fjsp_last_error.restype = ctypes.c_char_p
    return L


def chk(L, rc):
    if rc != 0:
        raise RuntimeError(L.fjsp_last_error().decode())


variants = []
for sp in specs:
    path, _, opt = sp.partition(":")
    L = open_lib(path)
    h = P()
    cfg = nat.default_config()
    chk(L, L.fjsp_create(ctypes.byref(cfg), N, 0, P(stream.cuda_stream), ctypes.byref(h)))
    nostatus = False
    for kv in filter(None, opt.split(",")):
        k, v = kv.split("=")
        if k == "nostatus":   # the launch without the status output stream
            nostatus = bool(int(v))
            continue
        chk(L, L.fjsp_set_option(h, k.encode(), int(v)))
    seeds = torch.arange(N, dtype=torch.int32, device="cuda")
    chk(L, L.fjsp_reset(h, P(seeds.data_ptr()), None, 30, None))
    buf = V.Buffers(K, N, torch.device("cuda"), infos=False)
    if nostatus:
        buf.status = None
    variants.append({"spec": sp, "L": L, "h": h, "buf": buf, "t": 0, "ms": []})

first = []
for v in variants:   # warm-up launch, kept for the byte comparison
    chk(v["L"], v["L"].fjsp_step_many(v["h"], K, 1234, 0, v["t"], 0, 1, ctypes.byref(v["buf"].struct())))
    v["t"] += K
    torch.cuda.synchronize()
    first.append({k: x.copy() for k, x in __import__("tests.gpu_util", fromlist=["to_np"]).to_np(v["buf"]).items()})
for r in range(REPS):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        chk(v["L"], v["L"].fjsp_step_many(v["h"], K, 1234, 0, v["t"], 0, 1, ctypes.byref(v["buf"].struct())))
        e1.record(stream)
        torch.cuda.synchronize()
        v["t"] += K
        v["ms"].append(e0.elapsed_time(e1))
out = {"N": N, "K": K, "reps": REPS, "variants": []}
for i, v in enumerate(variants):
    same = all(first[i][k].tobytes() == first[0][k].tobytes() for k in first[0] if k in first[i])
    out["variants"].append({"spec": v["spec"], "median_ms": float(np.median(v["ms"])), "mean_ms": float(np.mean(v["ms"])),
                            "min_ms": float(np.min(v["ms"])), "us_per_step_median": float(np.median(v["ms"])) * 1e3 / K,
                            "bytes_equal_to_first": same})
print(json.dumps(out))
