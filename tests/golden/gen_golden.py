"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

TEST INFRASTRUCTURE — runs only in the build container (it imports /root/reference, which
does not exist on the GPU box).  The reference's missing third-party modules (simpy,
gymnasium, pettingzoo; requirements.txt:6-8) are replaced by the stand-ins in
``tests/golden/standins``; ``visualization`` (matplotlib TkAgg,
visualization.py:13) is stubbed because a2c.py imports it and tkinter is absent.

Outputs (all small, committed):
  reset_tables.npz  — order tables (n_products, type, colour) for seeds 0..255 and for
                      seed-continued resets (reference FJSPSimulation.py:101-131,286-323).
  traces.npz        — full step traces (actions, obs, rewards, term, trunc, infos,
                      action results, reset obs) for seeds 0..3 x {unmasked, masked,
                      heuristic(2 orders)} x 1000 steps with auto-reset
                      (FJSPSimulation.py:144-242; a2c.py:390-537 for the heuristic).
  digests.json      — sha256 digests of 50-step chunks of the canonical per-env record for
                      256 envs x 1000 unmasked-random steps (env i seeded i).
  scenarios.npz     — scripted traces with non-default configs (storage capacity 2, tray
                      capacity 3) and hand-written action scripts hitting the edge paths.
  heur_probe.npz    — mixed heuristic / masked-random rollouts recording, at every step, the
                      heuristic's proposal (a2c.py:390-537) and a2c's flattened global state
                      (a2c.py:118-166) for the pre-step observation.
  gae.npz           — returns/advantages from transition_memory.MultiAgentTransitionMemory
                      (transition_memory.py:45-105) on recorded reward streams.

Actions for the random policies come from the counter RNG spec shared with the oracle and
the HIP kernel (``action_rng`` below).

Usage:  python tests/golden/gen_golden.py [--quick]
"""
import argparse
import contextlib
import hashlib
import io
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

AGENTS = ["pickup_station", "agv", "small_machine", "big_machine",
          "packaging_blue_1", "packaging_blue_2", "packaging_red", "packaging_green"]
N_ACTIONS = [3, 8, 3, 3, 3, 3, 3, 3]
# bit order of the per-agent action-result word (reference result dicts:
# PickupStationAgent.py:198-204, AGVAgent.py:196-205, MachineAgent.py:106-112,
# PackagingAgent.py:308-315). bit 7 = the agent executed an action this step.
RESULT_KEYS = {
    "pickup_station": ["success", "product_loaded", "tray_completed", "idle_with_orders"],
    "agv": ["success", "invalid_action", "moved", "pickup_success", "drop_success",
            "delivered_to_packaging"],
    "machine": ["success", "started_processing", "completed_processing", "idle_with_queue"],
    "packaging": ["success", "started_packaging", "completed_packaging", "idle_with_queue"],
}
RESULT_INT = {"agv": "distance", "packaging": "products_completed_this_step"}

M64 = (1 << 64) - 1


def fmix64(z):
    z &= M64
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    return z


def action_rng(seed, env_gid, step, masks=None):
    """Counter RNG for synthetic actions (same spec in oracle/fjsp_oracle.c and the kernel).

    h = fmix64(seed ^ fmix64((env_gid << 32) | step)); byte_a = (h >> 8a) & 0xFF;
    unmasked: a = byte*n >> 8; masked: j = byte*popcount(mask) >> 8, a = j-th set bit."""
    h = fmix64((seed & M64) ^ fmix64(((env_gid & 0xFFFFFFFF) << 32) | (step & 0xFFFFFFFF)))
    out = []
    for a in range(8):
        b = (h >> (8 * a)) & 0xFF
        if masks is None:
            out.append((b * N_ACTIONS[a]) >> 8)
        else:
            m = masks[a]
            bits = [i for i in range(len(m)) if m[i]]
            j = (b * len(bits)) >> 8
            out.append(bits[j])
    return out


def agent_kind(a):
    if a in ("small_machine", "big_machine"):
        return "machine"
    if a.startswith("packaging"):
        return "packaging"
    return a


def import_reference():
    sys.path.insert(0, os.path.join(HERE, "standins"))
    sys.path.insert(0, REF)
    viz = types.ModuleType("visualization")

    class GridVisualizer:  # a2c.py imports it; never used here
        def __init__(self, *a, **k):
            pass
    viz.GridVisualizer = GridVisualizer
    sys.modules["visualization"] = viz
    import FJSPParallelEnvWrapper  # noqa
    import a2c  # noqa
    import transition_memory  # noqa
    return FJSPParallelEnvWrapper, a2c, transition_memory


def flatten_obs(obs):
    """Canonical SoA record of one env's observation dict (agent order, key insertion order)."""
    i32, i8, f32, mask = [], [], [], []
    for a in AGENTS:
        for k, v in obs[a].items():
            if k == "action_mask":
                mask.extend(int(x) for x in v.reshape(-1))
            elif v.dtype == np.int32:
                i32.extend(int(x) for x in v.reshape(-1))
            elif v.dtype == np.int8:
                i8.append(int(v))
            elif v.dtype == np.float32:
                f32.append(np.float32(v))
            else:
                raise TypeError((a, k, v.dtype))
    return (np.array(i32, np.int32), np.array(i8, np.int8), np.array(f32, np.float32),
            np.array(mask, np.int8))


def encode_result(a, res):
    if not res:
        return 0
    kind = agent_kind(a)
    w = 1 << 7
    for bit, key in enumerate(RESULT_KEYS[kind]):
        if res.get(key, False):
            w |= 1 << bit
    if kind in RESULT_INT:
        w |= (int(res[RESULT_INT[kind]]) & 0xFFFF) << 16
    return w


def masks_of(obs):
    return [np.asarray(obs[a]["action_mask"]).astype(int).tolist() for a in AGENTS]


def run_trace(W, a2c_mod, seed, policy, steps, num_orders, config=None, script=None, rng_env=0):
    """Run one reference env for `steps` steps with auto-reset (seed=None, a2c.py:380)."""
    env = W.FJSPParallelEnv(config=config)
    np.random.seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        obs, _ = env.reset(seed=seed, options={"num_orders": num_orders})
    heur = None
    if policy == "heuristic":
        heur = a2c_mod.MultiAgentA2C.__new__(a2c_mod.MultiAgentA2C)
    rec = {k: [] for k in ["actions", "obs_i32", "obs_i8", "obs_f32", "masks", "rewards",
                           "term", "trunc", "sim_time", "orders_completed", "packaged",
                           "results", "reset_i32", "reset_i8", "reset_f32", "reset_masks"]}
    r0 = flatten_obs(obs)
    init = {"init_i32": r0[0], "init_i8": r0[1], "init_f32": r0[2], "init_masks": r0[3]}
    for t in range(steps):
        if policy == "unmasked":
            act = action_rng(seed, rng_env, t)
        elif policy == "masked":
            act = action_rng(seed, rng_env, t, masks_of(obs))
        elif policy == "heuristic":
            hd = heur._get_heuristic_actions(env.unwrapped.simulation)
            act = [hd[a] for a in AGENTS]
        elif policy == "script":
            act = script[t % len(script)]
        actions = {a: int(act[i]) for i, a in enumerate(AGENTS)}
        with contextlib.redirect_stdout(io.StringIO()):
            obs, rew, term, trunc, info = env.step(actions)
        f = flatten_obs(obs)
        rec["actions"].append(np.array(act, np.uint8))
        rec["obs_i32"].append(f[0]); rec["obs_i8"].append(f[1])
        rec["obs_f32"].append(f[2]); rec["masks"].append(f[3])
        rec["rewards"].append(np.array([rew[a] for a in AGENTS], np.float64))
        te = term[AGENTS[0]]; tr = trunc[AGENTS[0]]
        assert all(term[a] == te for a in AGENTS) and all(trunc[a] == tr for a in AGENTS)
        rec["term"].append(np.uint8(te)); rec["trunc"].append(np.uint8(tr))
        i0 = info[AGENTS[0]]
        rec["sim_time"].append(float(i0["sim_time"]))
        rec["orders_completed"].append(int(i0["orders_completed"]))
        rec["packaged"].append(int(i0["total_products_packaged"]))
        rec["results"].append(np.array([encode_result(a, info[a]["action_result"])
                                        for a in AGENTS], np.uint32))
        if te or tr:
            with contextlib.redirect_stdout(io.StringIO()):
                obs, _ = env.reset(options={"num_orders": num_orders})
            f = flatten_obs(obs)
        rec["reset_i32"].append(f[0]); rec["reset_i8"].append(f[1])
        rec["reset_f32"].append(f[2]); rec["reset_masks"].append(f[3])
    out = {k: np.stack(v) if isinstance(v[0], np.ndarray) else np.array(v) for k, v in rec.items()}
    out.update(init)
    return out


def record_bytes(tr, t):
    """Canonical per-step record used by the digests (see tests/parity_util.py)."""
    return b"".join([tr["obs_i32"][t].tobytes(), tr["obs_i8"][t].tobytes(),
                     tr["obs_f32"][t].tobytes(), tr["masks"][t].tobytes(),
                     tr["rewards"][t].tobytes(), bytes([tr["term"][t], tr["trunc"][t]])])


def gen_reset_tables(W):
    env = W.FJSPParallelEnv()
    tabs = np.zeros((256, 30, 3), np.uint8)
    for s in range(256):
        with contextlib.redirect_stdout(io.StringIO()):
            env.reset(seed=s, options={"num_orders": 30})
        for i, o in enumerate(env.simulation.orders):
            tabs[s, i] = (len(o.products), o.products[0].product_type.value,
                          o.products[0].packaging_color.value)
    # continued stream: seed s, then 3 resets with seed=None and 25 orders
    cont = np.zeros((16, 4, 25, 3), np.uint8)
    for s in range(16):
        for r in range(4):
            with contextlib.redirect_stdout(io.StringIO()):
                env.reset(seed=s if r == 0 else None, options={"num_orders": 25})
            for i, o in enumerate(env.simulation.orders):
                cont[s, r, i] = (len(o.products), o.products[0].product_type.value,
                                 o.products[0].packaging_color.value)
    np.savez_compressed(os.path.join(HERE, "reset_tables.npz"), seeded=tabs, continued=cont)


def gen_traces(W, a2c_mod, steps):
    out = {}
    for seed in range(4):
        for policy, norders in (("unmasked", 30), ("masked", 30), ("heuristic", 2)):
            tr = run_trace(W, a2c_mod, seed, policy, steps, norders, rng_env=seed)
            for k, v in tr.items():
                out[f"{policy}_s{seed}_{k}"] = v
    np.savez_compressed(os.path.join(HERE, "traces.npz"), **out)


def gen_digests(W, a2c_mod, n_envs, steps, chunk=50):
    dig = {"n_envs": n_envs, "steps": steps, "chunk": chunk, "num_orders": 30,
           "policy": "unmasked", "action_seed": 0, "digests": []}
    for e in range(n_envs):
        # env e is seeded e; actions keyed by (action_seed=0, env_gid=e, step)
        env = W.FJSPParallelEnv()
        with contextlib.redirect_stdout(io.StringIO()):
            env.reset(seed=e, options={"num_orders": 30})
        tr = run_trace_rngseed(W, env, e, steps)
        row = []
        for c in range(0, steps, chunk):
            h = hashlib.sha256()
            for t in range(c, min(steps, c + chunk)):
                h.update(record_bytes(tr, t))
            row.append(h.hexdigest()[:16])
        dig["digests"].append(row)
        if e % 32 == 0:
            print("digest env", e, flush=True)
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(dig, f)


def run_trace_rngseed(W, env, e, steps, num_orders=30):
    rec = {k: [] for k in ["obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc"]}
    for t in range(steps):
        act = action_rng(0, e, t)
        actions = {a: int(act[i]) for i, a in enumerate(AGENTS)}
        with contextlib.redirect_stdout(io.StringIO()):
            obs, rew, term, trunc, info = env.step(actions)
        f = flatten_obs(obs)
        rec["obs_i32"].append(f[0]); rec["obs_i8"].append(f[1])
        rec["obs_f32"].append(f[2]); rec["masks"].append(f[3])
        rec["rewards"].append(np.array([rew[a] for a in AGENTS], np.float64))
        te = term[AGENTS[0]]; tr = trunc[AGENTS[0]]
        rec["term"].append(int(te)); rec["trunc"].append(int(tr))
        if te or tr:
            with contextlib.redirect_stdout(io.StringIO()):
                env.reset(options={"num_orders": num_orders})
    return rec


# Hand-written action scripts (one row = one step, agent order) exercising edge paths.
# S = stay idle row.
IDLE = [0, 0, 0, 0, 0, 0, 0, 0]


def scenario_scripts():
    sc = {}
    # 1) load a full order onto trays, ship through the small machine to packaging,
    #    hitting the boundary rule for machine (60) and packaging (30) completions.
    s = []
    s += [[1, 0, 0, 0, 0, 0, 0, 0]] * 6          # pickup loads products
    s += [[2, 0, 0, 0, 0, 0, 0, 0]]              # signal partial tray
    s += [[0, 6, 0, 0, 0, 0, 0, 0]]              # AGV picks up at pickup
    s += [[0, 2, 0, 0, 0, 0, 0, 0]]              # move to small machine
    s += [[0, 7, 1, 0, 0, 0, 0, 0]]              # drop + START in the same step
    s += [IDLE] * 3
    s += [[0, 3, 1, 1, 1, 1, 1, 1]]              # START while busy (refused) + moves
    s += [IDLE] * 40
    s += [[0, 2, 2, 0, 0, 0, 0, 0]]              # SIGNAL done
    s += [[0, 6, 0, 0, 0, 0, 0, 0]]              # pick up processed tray
    s += [[0, 5, 0, 0, 0, 0, 0, 0]]              # move to packaging
    s += [[0, 7, 0, 0, 1, 1, 1, 1]]              # drop + START everything
    s += [IDLE] * 2
    s += [[0, 0, 0, 0, 2, 2, 2, 2]]              # SIGNAL while busy
    s += [IDLE] * 3
    s += [[0, 0, 0, 0, 2, 2, 2, 2]]              # SIGNAL after completion (re-earnable)
    s += [[0, 0, 0, 0, 2, 2, 2, 2]]
    sc["pipeline"] = s
    # 2) storage round trips (with storage capacity 2 -> trays are lost at the 3rd drop)
    s = []
    for _ in range(4):
        s += [[1, 0, 0, 0, 0, 0, 0, 0], [2, 0, 0, 0, 0, 0, 0, 0]]
        s += [[0, 6, 0, 0, 0, 0, 0, 0], [0, 4, 0, 0, 0, 0, 0, 0], [0, 7, 0, 0, 0, 0, 0, 0],
              [0, 1, 0, 0, 0, 0, 0, 0]]
    s += [[0, 4, 0, 0, 0, 0, 0, 0], [0, 6, 0, 0, 0, 0, 0, 0], [0, 6, 0, 0, 0, 0, 0, 0],
          [0, 7, 0, 0, 0, 0, 0, 0], [0, 6, 0, 0, 0, 0, 0, 0], [0, 7, 0, 0, 0, 0, 0, 0],
          [0, 0, 0, 0, 0, 0, 0, 0], [0, 1, 0, 0, 0, 0, 0, 0], [0, 7, 0, 0, 0, 0, 0, 0],
          [0, 6, 0, 0, 0, 0, 0, 0]]
    sc["storage"] = s
    # 3) machine overwrite: start a second tray while the first is unsignalled, plus
    #    invalid / out-of-range actions for every agent.
    s = []
    s += [[1, 0, 0, 0, 0, 0, 0, 0]] * 3 + [[2, 0, 0, 0, 0, 0, 0, 0]]
    s += [[1, 0, 0, 0, 0, 0, 0, 0]] * 2 + [[2, 0, 0, 0, 0, 0, 0, 0]]
    s += [[0, 6, 0, 0, 0, 0, 0, 0], [0, 2, 0, 0, 0, 0, 0, 0], [0, 7, 0, 0, 0, 0, 0, 0],
          [0, 3, 0, 0, 0, 0, 0, 0], [0, 7, 0, 0, 0, 0, 0, 0], [0, 1, 0, 0, 0, 0, 0, 0],
          [0, 6, 0, 0, 0, 0, 0, 0], [0, 2, 1, 1, 0, 0, 0, 0], [0, 7, 0, 0, 0, 0, 0, 0]]
    s += [[0, 9, 7, 5, 4, 9, 3, 200]] * 2
    s += [IDLE] * 25
    s += [[0, 0, 1, 1, 0, 0, 0, 0]]   # start again while unsignalled -> overwrite
    s += [IDLE] * 20
    s += [[0, 0, 2, 2, 0, 0, 0, 0]] + [[1, 7, 0, 0, 0, 0, 0, 0]]
    sc["overwrite"] = s
    return sc


def gen_scenarios(W, a2c_mod):
    out = {}
    base = {'num_trays': 1000, 'tray_capacity': 5, 'num_packaging_blue': 2, 'num_packaging_red': 1,
            'num_packaging_green': 1, 'grid_rows': 4, 'grid_cols': 6, 'agv_speed': 1,
            'step_size': 10, 'max_episode_steps': 200}
    cfgs = {
        "pipeline": dict(base),
        "storage": dict(base, storage_capacity=2),
        "overwrite": dict(base, tray_capacity=3),
    }
    for name, script in scenario_scripts().items():
        for seed in (0, 7):
            tr = run_trace(W, a2c_mod, seed, "script", len(script) + 10, 5,
                           config=cfgs[name], script=script + [IDLE] * 10)
            for k, v in tr.items():
                out[f"{name}_s{seed}_{k}"] = v
    # short episodes: max_episode_steps=30, heuristic with 1 order (terminates) and
    # masked random (truncates) -> auto-reset paths with a non-default truncation limit
    for seed in (3, 11):
        cfg = dict(base, max_episode_steps=30)
        tr = run_trace(W, a2c_mod, seed, "heuristic", 150, 1, config=cfg)
        for k, v in tr.items():
            out[f"short_heur_s{seed}_{k}"] = v
    np.savez_compressed(os.path.join(HERE, "scenarios.npz"), **out)


def gen_heur_probe(W, a2c_mod, steps=400, seeds=range(6)):
    """States reached by a mix of heuristic and masked-random actions (the heuristic alone
    never drops at storage: it compares the AGV position with (1, 5), constants.py:9 puts
    STORAGE at (3, 0)), with the heuristic's proposal and a2c's global state at each step."""
    out = {}
    agent = a2c_mod.MultiAgentA2C.__new__(a2c_mod.MultiAgentA2C)
    env0 = W.FJSPParallelEnv()
    agent.possible_agents = list(env0.possible_agents)
    agent.obs_dims = {a: agent._get_obs_dim(env0.observation_space(a)) for a in AGENTS}
    for seed in seeds:
        env = W.FJSPParallelEnv()
        np.random.seed(seed)
        with contextlib.redirect_stdout(io.StringIO()):
            obs, _ = env.reset(seed=seed, options={"num_orders": 30})
        acts, heur, gs = [], [], []
        for t in range(steps):
            hd = agent._get_heuristic_actions(env.unwrapped.simulation)
            h = [int(hd[a]) for a in AGENTS]
            gs.append(agent._get_global_state(obs, list(env.agents)).astype(np.float32))
            use_h = (fmix64(seed * 7919 + t) >> 11) % 3 != 0
            act = h if use_h else action_rng(seed + 100, seed, t, masks_of(obs))
            with contextlib.redirect_stdout(io.StringIO()):
                obs, rew, term, trunc, info = env.step({a: int(act[i]) for i, a in enumerate(AGENTS)})
                if term[AGENTS[0]] or trunc[AGENTS[0]]:
                    obs, _ = env.reset(options={"num_orders": 30})
            acts.append(np.array(act, np.uint8))
            heur.append(np.array(h, np.uint8))
        out[f"s{seed}_actions"] = np.stack(acts)
        out[f"s{seed}_heur"] = np.stack(heur)
        out[f"s{seed}_gstate"] = np.stack(gs)
    np.savez_compressed(os.path.join(HERE, "heur_probe.npz"), **out)


def gen_gae(tm_mod):
    rng = np.random.default_rng(1234)
    cases = {}
    for ci, (T, segs, gamma, lamb) in enumerate([(64, [17, 64], 0.99, 0.95),
                                                   (256, [1, 100, 201, 256], 0.99, 0.99),
                                                   (37, [37], 0.9, 0.5)]):
        rewards = np.round(rng.normal(0, 3, size=(T, 8)) * 8) / 8  # like env rewards
        values = rng.normal(0, 5, size=(T, 8)).astype(np.float32)
        # a2c semantics: episode ends bootstrap with 0.0 (a2c.py:357-358), the batch end with
        # the critic's V(s) (a2c.py:324-332)
        boots = rng.normal(0, 5, size=(len(segs), 8)).astype(np.float32)
        boots[:-1] = 0.0
        mem = tm_mod.MultiAgentTransitionMemory(AGENTS, gamma, lamb, True)
        start = 0
        for si, end in enumerate(segs):
            for t in range(start, end):
                mem.put({a: None for a in AGENTS}, {a: 0 for a in AGENTS},
                        {a: float(rewards[t, i]) for i, a in enumerate(AGENTS)},
                        {a: None for a in AGENTS},
                        {a: float(values[t, i]) for i, a in enumerate(AGENTS)})
            mem.finish_trajectory({a: float(boots[si, i]) for i, a in enumerate(AGENTS)})
            start = end
        ret = np.array([mem.return_lst[a] for a in AGENTS]).T
        adv = np.array([mem.adv_lst[a] for a in AGENTS]).T
        seg_end = np.zeros(T, np.uint8)
        for e in segs:
            seg_end[e - 1] = 1
        cases[f"c{ci}_rewards"] = rewards
        cases[f"c{ci}_values"] = values
        cases[f"c{ci}_boots"] = boots
        cases[f"c{ci}_seg_end"] = seg_end
        cases[f"c{ci}_gamma_lamb"] = np.array([gamma, lamb])
        cases[f"c{ci}_returns"] = ret
        cases[f"c{ci}_adv"] = adv
    np.savez_compressed(os.path.join(HERE, "gae.npz"), **cases)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    W, a2c_mod, tm_mod = import_reference()
    only = set(args.only.split(",")) if args.only else None

    def want(x):
        return only is None or x in only
    if want("reset"):
        gen_reset_tables(W)
    if want("gae"):
        gen_gae(tm_mod)
    if want("heur_probe"):
        gen_heur_probe(W, a2c_mod)
    if want("scenarios"):
        gen_scenarios(W, a2c_mod)
    if want("traces"):
        gen_traces(W, a2c_mod, 200 if args.quick else 1000)
    if want("digests"):
        gen_digests(W, a2c_mod, 8 if args.quick else 256, 1000)


if __name__ == "__main__":
    main()
