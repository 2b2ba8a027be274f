"""Golden vectors for the reference's TRAINED policy (/root/reference/checkpoints/model.pt).

TEST INFRASTRUCTURE — runs only in the build container (imports /root/reference through
gen_golden.import_reference; the checkpoint does not travel, its weights do, as data).

The checkpoint is read with the package's weights-only loader
(a2c_vec.load_checkpoint: torch.load(weights_only=True) with an allowlist of exactly the numpy
scalar global and the int64 dtype class that a2c.py:80 pickles into act_dims) — never with the
reference's own weights_only=False load (a2c.py:767).  Its state dicts are then loaded into the
reference's MultiAgentA2C networks exactly as load_model does (a2c.py:770-773), and the
reference's own test() loop (a2c.py:539-645: reset, predict(deterministic=True), step until
env.agents is empty or max_steps) is run per seed, recording at every step the pre-step
observation as the a2c features (_get_global_state, a2c.py:136-166) and masks, the reference's
greedy actions and critic value, and each agent's top-2 masked-probability margin (a2c.py:204-229)
so that the consumer can tell a genuine mismatch from an f32 near-tie.

Output trained_policy.npz:
  w_actor.<agent>.<param>, w_critic.<param>   f32 trained weights (the checkpoint's tensors)
  s<seed>_gstate [T, 38] f32, s<seed>_masks [T, 29] i8, s<seed>_actions [T, 8] u8,
  s<seed>_values [T] f32, s<seed>_margin [T, 8] f32, s<seed>_rewards [T, 8] f64,
  s<seed>_meta = [num_orders, steps, orders_completed, products_packaged]
"""
import contextlib
import importlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
import gen_golden as GG  # noqa: E402

CKPT = "/root/reference/checkpoints/model.pt"
CASES = [(0, 5), (1, 5), (2, 5), (3, 5), (4, 25), (5, 25), (6, 2), (7, 2)]   # (seed, num_orders)
MAX_STEPS = 500


def main():
    import torch
    A = importlib.import_module("multi-agent-rl-for-fjsp_amd.a2c_vec")
    ck = A.load_checkpoint(CKPT)
    W, a2c_mod, _ = GG.import_reference()
    os.chdir("/tmp")
    out = {}
    for a, sd in ck["actor_nets"].items():
        for k, v in sd.items():
            out[f"w_actor.{a}.{k}"] = v.numpy().astype(np.float32)
    for k, v in ck["critic_net"].items():
        out[f"w_critic.{k}"] = v.numpy().astype(np.float32)

    for seed, num_orders in CASES:
        env = W.FJSPParallelEnv()
        agent = a2c_mod.MultiAgentA2C(env)
        for a, sd in ck["actor_nets"].items():            # load_model, a2c.py:770-773
            agent.actor_nets[a].load_state_dict(sd)
        agent.critic_net.load_state_dict(ck["critic_net"])
        np.random.seed(seed)
        with contextlib.redirect_stdout(io.StringIO()):
            obs, _ = env.reset(seed=seed, options={"num_orders": num_orders})
        rec = {k: [] for k in ("gstate", "masks", "actions", "values", "margin", "rewards")}
        steps, oc, pk = 0, 0, 0
        while env.agents and steps < MAX_STEPS:           # test(), a2c.py:583-620
            active = list(env.agents)
            rec["gstate"].append(agent._get_global_state(obs, active).astype(np.float32))
            rec["masks"].append(np.concatenate([np.asarray(obs[a]["action_mask"], np.int8) for a in GG.AGENTS]))
            with torch.no_grad():
                acts, _, vals = agent.predict(obs, active, train_returns=True, deterministic=True)
                margin = []
                for a in GG.AGENTS:                        # the masked probabilities of a2c.py:200-220
                    p = agent.actor_nets[a](torch.FloatTensor(agent._flatten_obs(obs[a])))
                    m = torch.tensor(obs[a]["action_mask"], dtype=torch.float32)
                    p = p * m
                    p = p / p.sum() if p.sum() > 0 else m / m.sum()
                    top = torch.sort(p, descending=True).values
                    margin.append(float(top[0] - top[1]) if top.numel() > 1 else 1.0)
            rec["actions"].append(np.array([acts[a] for a in GG.AGENTS], np.uint8))
            rec["values"].append(np.float32(vals[GG.AGENTS[0]].reshape(-1)[0]))
            rec["margin"].append(np.array(margin, np.float32))
            with contextlib.redirect_stdout(io.StringIO()):
                obs, rew, term, trunc, infos = env.step(acts)
            rec["rewards"].append(np.array([rew[a] for a in GG.AGENTS], np.float64))
            for info in infos.values():
                oc = info.get("orders_completed", oc)
                pk = info.get("total_products_packaged", pk)
            steps += 1
        for k, v in rec.items():
            out[f"s{seed}_{k}"] = np.stack(v)
        out[f"s{seed}_meta"] = np.array([num_orders, steps, oc, pk], np.int64)
        print(f"seed {seed} orders {num_orders}: {steps} steps, {oc} orders, {pk} products, "
              f"min margin {out[f's{seed}_margin'].min():.3g}, action hist "
              f"{[np.bincount(out[f's{seed}_actions'][:, i], minlength=3).tolist() for i in range(8)]}")
    np.savez_compressed(os.path.join(HERE, "trained_policy.npz"), **out)


if __name__ == "__main__":
    main()
