"""A/B of the one-launch-per-step kernel (k_step<canon>, fjsp_step with host-supplied actions, the
reference-API path) between library builds: N envs, interleaved rounds of 200 launches, HIP-event
time per launch (median of rounds), outputs of the first round byte-compared.

usage: python scripts/ab_kstep.py [N] [rounds] lib[:option=value] ...  (e.g. libfjsp.so:step_envs=16)"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import importlib  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402

nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 6
specs = sys.argv[3:]
P = ctypes.c_void_p
stream = torch.cuda.current_stream()
variants = []
for spec in specs:
    path, _, opt = spec.partition(":")
    L = ctypes.CDLL(os.path.abspath(path))
    L.fjsp_create.argtypes = [ctypes.POINTER(nat.fjsp_config), ctypes.c_int32, ctypes.c_int32, P, ctypes.POINTER(P)]
    L.fjsp_reset.argtypes = [P, P, P, ctypes.c_int32, ctypes.POINTER(nat.fjsp_out)]
    L.fjsp_step.argtypes = [P, P, P, ctypes.c_int32, ctypes.POINTER(nat.fjsp_out)]
    L.fjsp_set_option.argtypes = [P, ctypes.c_char_p, ctypes.c_int64]
    h = P()
    cfg = nat.default_config()
    assert L.fjsp_create(ctypes.byref(cfg), N, 0, P(stream.cuda_stream), ctypes.byref(h)) == 0
    assert L.fjsp_set_option(h, b"timing", 0) == 0
    if opt:
        k, val = opt.split("=")
        assert L.fjsp_set_option(h, k.encode(), int(val)) == 0, opt
    seeds = torch.arange(N, dtype=torch.int32, device="cuda")
    assert L.fjsp_reset(h, P(seeds.data_ptr()), None, 30, None) == 0
    buf = V.Buffers(1, N, torch.device("cuda"), infos=False)
    variants.append({"spec": spec, "L": L, "h": h, "buf": buf, "ms": []})
g = torch.Generator(device="cuda").manual_seed(5)
acts = [torch.randint(0, 3, (8, N), dtype=torch.uint8, device="cuda", generator=g) for _ in range(200)]
first = []
for r in range(ROUNDS + 1):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        o = v["buf"].struct()
        e0.record(stream)
        for a in acts:
            assert v["L"].fjsp_step(v["h"], P(a.data_ptr()), None, 1, ctypes.byref(o)) == 0
        e1.record(stream)
        torch.cuda.synchronize()
        if r == 0:
            b = v["buf"]
            first.append(b"".join(t.cpu().numpy().tobytes() for t in (b.rewards, b.obs_i32, b.obs_i8, b.obs_f32, b.masks,
                                                                       b.term, b.trunc)))
        else:
            v["ms"].append(e0.elapsed_time(e1) / len(acts))
out = {"N": N, "launches_per_round": len(acts), "rounds": ROUNDS,
       "variants": [{"spec": v["spec"], "median_ms_per_launch": float(np.median(v["ms"])),
                     "bytes_equal_to_first": first[i] == first[0]} for i, v in enumerate(variants)]}
print(json.dumps(out))
