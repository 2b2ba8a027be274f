"""k_policy (fjsp_a2c_policy) time at N envs in the library FJSP_LIB selects: HIP events around
100 launches on synthetic features / masks (random-init networks).

usage: FJSP_LIB=... python scripts/diag_policy.py [N]
"""
import ctypes
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda")
actors, critic = A.init_networks(seed=0, device=dev)
pa, pc = A.pack_policy_weights(actors, critic)
g = torch.Generator(device=dev).manual_seed(1)
feats = torch.randint(0, 5, (38, N), device=dev, generator=g).float()
masks = torch.ones(29, N, dtype=torch.int8, device=dev)
seed = torch.tensor([7], dtype=torch.int64, device=dev)
act = torch.empty(8, N, dtype=torch.uint8, device=dev)
val = torch.empty(N, dtype=torch.float32, device=dev)
stream = torch.cuda.current_stream()
P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731


def call(t):
    nat.check(nat.lib().fjsp_a2c_policy(P(feats), P(masks), N, P(pa), P(pc), P(seed), 0, t, 0, P(act), P(val), None,
                                        ctypes.c_void_p(stream.cuda_stream)))


for t in range(10):
    call(t)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(stream)
for t in range(100):
    call(t)
e1.record(stream)
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 10.0
with torch.no_grad():
    pm, v = A.masked_probs(actors(A.actor_inputs(feats, A.gather_index(dev))), A.agent_masks(masks, A.mask_index(dev))), \
        critic(feats.t()).view(-1)
    out = torch.empty(8, 8, N, device=dev)
    nat.check(nat.lib().fjsp_a2c_policy(P(feats), P(masks), N, P(pa), P(pc), P(seed), 0, 0, 1, P(act), P(val), P(out),
                                        ctypes.c_void_p(stream.cuda_stream)))
    torch.cuda.synchronize()
print(json.dumps({"lib": os.path.basename(nat.LIB_PATH), "N": N, "us_per_launch": us,
                  "tflops": 2 * 675e3 * N / (us * 1e-6) / 1e12,
                  "max_prob_err": float((out - pm).abs().max()), "max_value_err": float((val - v).abs().max())}))
