"""Where the grouped (dedup) A2C update spends its time at N envs x 256 steps: update_step's
stages run one after another with a device synchronisation between them (wall ms per stage,
median of 3 updates after a warm-up).

usage: python scripts/diag_update_stages.py [N]
"""
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
ve = importlib.import_module("multi-agent-rl-for-fjsp_amd.vec_env")
D = importlib.import_module("multi-agent-rl-for-fjsp_amd.distributed")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096

env = ve.FJSPVecEnv(N)
L = A.VecMultiAgentA2C(env, seed=0, dedup=True)
L.reset(seeds=torch.arange(N), num_orders=25)
L.collect()
ret, adv = L.advantages()
b = L._bufs
T = L.batch_size
print("optimizer defaults:", L.optim_actor.defaults.get("fused"), file=sys.stderr)
feats, masks, actions = b["feats"][:T], b["masks"][:T], b["actions"]


def run(st):
    t = [time.perf_counter()]

    def mark(name):
        torch.cuda.synchronize()
        now = time.perf_counter()
        st.setdefault(name, []).append((now - t[0]) * 1e3)
        t[0] = now
    S = T * N
    adv32 = adv.float().permute(1, 0, 2).reshape(A.NA, S)
    ret32 = ret.float().permute(1, 0, 2).reshape(A.NA, S)
    acts = actions.long().permute(1, 0, 2).reshape(A.NA, S)
    count, mean, std = D.adv_stats(adv32, None)
    L.optim_actor.zero_grad(set_to_none=True)
    L.optim_critic.zero_grad(set_to_none=True)
    mark("prep+adv_stats")
    gt = feats.permute(1, 0, 2).reshape(A.GLOBAL_DIM, S)
    f3 = feats.contiguous()
    mark("critic_T")
    keys = A.group_keys(f3)
    mark("group_keys")
    gr = A.RowGroups(keys)
    ga, gc = gr.rows(0, A.NA), gr.rows(A.NA, A.NA + 1)
    mark("RowGroups")
    assert A.group_verify(f3, ga, gc)
    mark("verify")

    def cols(agents, idx):
        k, u = idx.shape
        c = gt[:, idx.reshape(-1)].view(A.GLOBAL_DIM, k, u)
        c = torch.cat([c, c.new_zeros(1, k, u)])
        return c[L.gidx[agents], torch.arange(k, device=idx.device)[:, None], :]
    adv_n = (adv32 - mean[:, None]) / (std[:, None] + 1e-8)
    pu = L.actors.forward_rows(None, ga, cols)
    mark("actor_forward_rows")
    al = A._ActorHead.apply(pu, ga, masks.contiguous(), b["actions"].contiguous(), adv.contiguous(), mean, std,
                            float(count), L.entropy_coef)
    mark("actor_head")
    vu = A.mlp_forward(L.critic.net, gt[:, gc.first[0]].t()).reshape(1, 1, -1)
    v = gc.gather(vu).reshape(-1)
    cl = ((v[None, :] - ret32) ** 2).sum() / (A.NA * count)
    mark("critic_forward+loss")
    cl.backward()
    mark("backward_critic")
    al.sum().backward()
    mark("backward_actors")
    A.clip_per_agent_(L.actors, L.max_grad_norm)
    torch.nn.utils.clip_grad_norm_(L.critic.parameters(), L.max_grad_norm)
    L.optim_actor.step()
    L.optim_critic.step()
    mark("clip+adam")
    al.cpu(), cl.cpu()
    L.repack()
    mark("losses+repack")
    return ga.U, gc.U


st = {}
run({})
for _ in range(3):
    U = run(st)
med = {k: round(float(np.median(v)), 3) for k, v in st.items()}
med["total"] = round(sum(med.values()), 3)
print(json.dumps({"N": N, "samples": T * N, "groups_actors": U[0], "groups_critic": U[1], "stage_ms": med}))

# the same update unsynchronised (VecMultiAgentA2C.update), with and without the GAE pass
tt = {"update_given_adv": [], "update_with_gae": [], "gae_only": []}
for _ in range(3):
    for key, fn in (("update_given_adv", lambda: L.update(ret, adv)), ("update_with_gae", lambda: L.update()),
                    ("gae_only", lambda: L.advantages())):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        tt[key].append((time.perf_counter() - t0) * 1e3)
print(json.dumps({k: round(float(np.median(v)), 3) for k, v in tt.items()}))
