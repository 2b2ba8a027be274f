"""A/B timing of the fused policy kernel (fjsp_a2c_policy) on the observations of a real A2C
collect: a 4 096-env learner collects one 256-step batch (random-init or the reference's
trained weights), then each library's kernel runs on those 256 (features, masks) slabs in
turn, HIP events per launch; outputs (greedy actions, values, probabilities) compared byte for
byte with the first library's.  Libraries through raw ctypes (the signature is unchanged since
ABI 3).

usage: python scripts/ab_policy.py [N] [init] lib[:order[:all|actors|values]] ...   (order -> FJSP_POLICY_ORDER)
"""
import ctypes
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

nat = importlib.import_module("multi-agent-rl-for-fjsp_amd._native")
A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
V = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
INIT = sys.argv[2] if len(sys.argv) > 2 else "random"
libs = sys.argv[3:] or [nat.LIB_PATH]
P = ctypes.c_void_p
stream = torch.cuda.current_stream()

L = A.VecMultiAgentA2C(V.FJSPVecEnv(N), batch_size=256, seed=0)
if INIT == "trained":
    L.load_state_dicts(A.load_npz_weights(os.path.join(REPO, "tests", "golden", "trained_policy.npz")))
L.reset(seeds=torch.arange(N), num_orders=25)
L.collect()
L.update()
L.roll_over()
L.collect()
torch.cuda.synchronize()
feats, masks = L._bufs["feats"], L._bufs["masks"]
T = L.batch_size

res = {"N": N, "init": INIT, "steps": T, "libs": []}
ref = None
for spec in libs:
    path, _, rest = spec.partition(":")
    order, _, part = rest.partition(":")
    part = part or "all"
    if order:
        os.environ["FJSP_POLICY_ORDER"] = order
    else:
        os.environ.pop("FJSP_POLICY_ORDER", None)
    lib = ctypes.CDLL(os.path.abspath(path))
    f = lib.fjsp_a2c_policy
    f.argtypes = [P, P, ctypes.c_int32, P, P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32, P, P, P, P]
    act = torch.zeros(8, N, dtype=torch.uint8, device="cuda")
    val = torch.zeros(N, dtype=torch.float32, device="cuda")
    probs = torch.zeros(8, 8, N, dtype=torch.float32, device="cuda")

    def run(t, det, pr=None):
        rc = f(P(feats[t].data_ptr()), P(masks[t].data_ptr()), N, P(L._pw_actor.data_ptr()), P(L._pw_critic.data_ptr()),
               P(L._rng.data_ptr()), 0, t, det, None if part == "values" else P(act.data_ptr()),
               None if part == "actors" else P(val.data_ptr()),
               None if pr is None or part == "values" else P(pr.data_ptr()), P(stream.cuda_stream))
        assert rc == 0
    outs = []
    for t in (0, 100, 255):
        run(t, 1, probs)
        torch.cuda.synchronize()
        outs.append((act.cpu().clone(), val.cpu().clone(), probs.cpu().clone()))
    for t in range(8):
        run(t, 0)
    ms = []
    for t in range(T):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run(t, 0)
        e1.record(stream)
        ms.append((e0, e1))
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) * 1e3 for a, b in ms]
    same = None
    if ref is None:
        ref = outs
    elif part == "all":
        same = all(torch.equal(a[i], b[i]) for a, b in zip(outs, ref) for i in range(3))
    res["libs"].append({"lib": spec, "median_us": float(np.median(ms)), "mean_us": float(np.mean(ms)),
                        "p10_us": float(np.percentile(ms, 10)), "p90_us": float(np.percentile(ms, 90)),
                        "outputs_equal_to_first": same})
print(json.dumps(res))
