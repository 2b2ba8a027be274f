"""GPU tests of the reference-API drop-in (FJSPParallelEnv / FJSPSimulation / transition_memory)
against the reference's golden traces: dict-level observations with the reference dtypes and
key order, Python-float rewards, bool term/trunc, decoded action-result infos, numpy global RNG
sharing, and the GAE drop-in."""
import importlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from tests import parity_util as P  # noqa: E402
from tests.golden.gen_golden import encode_result, flatten_obs  # noqa: E402

# key insertion order of the reference's observation dicts (PickupStationAgent.py:131-140,
# AGVAgent.py:60-75, MachineAgent.py:64-69, PackagingAgent.py:266-271)
REF_KEYS = {
    "pickup_station": ["order_size", "products_remaining", "next_product_type", "next_product_color",
                       "current_tray_type", "current_tray_color", "current_tray_count", "action_mask"],
    "agv": ["position", "carrying_tray", "tray_product_count", "tray_type", "tray_needs_processing",
            "tray_needs_packaging", "pickup_ready_trays", "small_machine_busy", "big_machine_busy",
            "small_machine_ready", "big_machine_ready", "storage_tray_count", "action_mask"],
}
STATION_KEYS = ["is_busy", "processing_progress", "queue_length", "action_mask"]


@pytest.fixture(scope="module")
def M():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from tests import gpu_util  # noqa: F401  (puts the repo on sys.path)
    return {
        "W": importlib.import_module("multi-agent-rl-for-fjsp_amd.FJSPParallelEnvWrapper"),
        "S": importlib.import_module("multi-agent-rl-for-fjsp_amd.FJSPSimulation"),
        "TM": importlib.import_module("multi-agent-rl-for-fjsp_amd.transition_memory"),
        "spec": importlib.import_module("multi-agent-rl-for-fjsp_amd.spec"),
    }


def _check_dict_obs(obs):
    for a, d in obs.items():
        keys = REF_KEYS.get(a, STATION_KEYS)
        assert list(d.keys()) == keys, a
        for k, v in d.items():
            assert isinstance(v, np.ndarray)
            if k == "action_mask":
                assert v.dtype == np.int8
            elif a in REF_KEYS:
                assert v.dtype == np.int32
            else:
                assert v.dtype == (np.float32 if k == "processing_progress" else np.int8)


@pytest.mark.parametrize("idx", range(0, 12, 2))
def test_parallel_env_replays_golden(M, idx):
    tr = P.load_traces()[idx]
    env = M["W"].FJSPParallelEnv()
    obs, infos = env.reset(seed=tr.seed, options={"num_orders": tr.num_orders})
    assert infos == {a: {} for a in env.possible_agents}
    _check_dict_obs(obs)
    f = flatten_obs(obs)
    assert P.bits_equal(f[0], tr.init_i32) and P.bits_equal(f[3], tr.init_masks)
    for t in range(tr.steps):
        actions = {a: int(tr.actions[t, i]) for i, a in enumerate(env.possible_agents)}
        obs, rew, term, trunc, info = env.step(actions)
        f = flatten_obs(obs)
        for j, k in enumerate(("obs_i32", "obs_i8", "obs_f32", "masks")):
            assert P.bits_equal(f[j], getattr(tr, k)[t]), (tr.name, t, k)
        assert all(type(r) is float for r in rew.values())
        assert P.bits_equal(np.array([rew[a] for a in env.possible_agents]), tr.rewards[t]), (tr.name, t)
        assert all(type(x) is bool for x in list(term.values()) + list(trunc.values()))
        assert term["agv"] == bool(tr.term[t]) and trunc["agv"] == bool(tr.trunc[t])
        for i, a in enumerate(env.possible_agents):
            assert encode_result(a, info[a]["action_result"]) == tr.results[t, i], (tr.name, t, a)
            assert info[a]["sim_time"] == tr.sim_time[t]
            assert info[a]["orders_completed"] == tr.orders_completed[t]
            assert info[a]["total_products_packaged"] == tr.packaged[t]
        # a2c.py:298-305 reads: taken from the observation, equal to the device state's AGV
        sim = env.unwrapped.simulation
        v = sim._venv.read_env(0)
        assert sim.agv.position == (v.agv_row, v.agv_col), (tr.name, t)
        ct = sim.agv.carrying_tray
        assert (ct is not None) == bool(v.agv_carrying), (tr.name, t)
        assert (len(ct) if ct is not None else 0) == v.agv_tray_count, (tr.name, t)
        if term["agv"] or trunc["agv"]:
            assert env.agents == []
            obs, _ = env.reset(options={"num_orders": tr.num_orders})    # seed=None: numpy stream continues
            f = flatten_obs(obs)
            assert P.bits_equal(f[0], tr.reset_i32[t]), (tr.name, t)
        else:
            assert env.agents == env.possible_agents
    _check_dict_obs(obs)


def test_global_numpy_stream_shared(M):
    """reset(seed=None) continues numpy's global MT19937 exactly like the reference (a2c.py:380)."""
    d = np.load(f"{P.GOLDEN}/reset_tables.npz")
    sim = M["S"].FJSPSimulation()
    for s in range(4):
        for r in range(4):
            sim.reset(seed=s if r == 0 else None, num_orders=25)
            det = sim.get_order_progress()["orders_detail"]
            got = np.array([[o["total_products"], 0, 0] for o in det], np.uint8)
            assert np.array_equal(got[:, 0], d["continued"][s, r, :, 0]), (s, r)
    # interleaving with other np.random users: state after reset == pure numpy emulation
    np.random.seed(77)
    np.random.random(13)
    exp = np.random.RandomState()
    exp.set_state(np.random.get_state())
    for _ in range(30):
        exp.randint(1, 10); exp.randint(0, 3); exp.randint(0, 3)
    sim.reset(num_orders=30)
    a, b = np.random.get_state(), exp.get_state()
    assert a[2] == b[2] and np.array_equal(a[1], b[1])


def test_order_progress_matches_oracle(M):
    sim = M["S"].FJSPSimulation()
    sim.reset(seed=3, num_orders=6)
    o = O.OracleEnv()
    o.reset(seed=3, num_orders=6)
    for t in range(180):
        acts = O.actions(1, 0, t, None)
        sim.step({a: int(acts[i]) for i, a in enumerate(M["spec"].AGENTS)})
        o.step(acts)
        if t % 30 == 29:
            prog = sim.get_order_progress()
            ow = o.orders()
            for i, dd in enumerate(prog["orders_detail"]):
                w = int(ow[i])
                assert (dd["total_products"], dd["processed"], dd["packaged"], dd["is_complete"]) == (
                    w & 15, (w >> 8) & 15, (w >> 12) & 15, bool((w >> 16) & 1))
            assert sim.current_step == t + 1


def test_dict_order_missing_and_odd_actions(M):
    """Actions dict in a non-canonical order, with missing agents, numpy / float / invalid values."""
    spec = M["spec"]
    sim = M["S"].FJSPSimulation()
    sim.reset(seed=9, num_orders=30)
    o = O.OracleEnv()
    o.reset(seed=9, num_orders=30)
    rng = np.random.default_rng(0)
    for t in range(300):
        order = rng.permutation(8)
        raw = O.actions(2, 5, t, None)
        actions, codes = {}, np.full(8, 255, np.uint8)
        for i in order:
            if rng.random() < 0.1:
                continue
            v = int(raw[i])
            u = rng.random()
            if u < 0.05:
                v, c = -1, 254
            elif u < 0.1:
                v, c = np.int64(v), v
            elif u < 0.13:
                v, c = float(v), v
            else:
                c = v
            actions[spec.AGENTS[i]] = v
            codes[i] = c
        present = [i for i in order if spec.AGENTS[i] in actions]
        full_order = present + [i for i in range(8) if i not in present]
        obs, rew, term, trunc, info = sim.step(actions)
        ro = o.step(codes, order=np.array(full_order, np.uint8))
        f = flatten_obs(obs)
        assert P.bits_equal(f[0], ro["obs_i32"]) and P.bits_equal(f[3], ro["masks"]), t
        assert P.bits_equal(np.array([rew[a] for a in spec.AGENTS]), ro["rewards"]), t
        for i, a in enumerate(spec.AGENTS):
            if a not in actions:
                assert info[a]["action_result"] == {}
        if term["agv"] or trunc["agv"]:
            sim.reset(num_orders=30)
            o.reset(num_orders=30)


def test_reward_weights_follow_reward_model(M):
    spec = M["spec"]
    sim = M["S"].FJSPSimulation()
    rm = sim.reward_calculator
    for k in ("ORDER_COMPLETE_REWARD", "THROUGHPUT_BONUS", "TIME_PENALTY", "AGV_INVALID_ACTION",
              "PACKAGING_COMPLETE_REWARD", "MACHINE_IDLE_PENALTY", "PICKUP_LOAD_REWARD"):
        setattr(rm, k, getattr(rm, k) * 1.37 + 0.011)
    sim.reset(seed=1, num_orders=3)
    prev_orders = prev_pk = 0
    for t in range(400):
        if t == 150:   # a weight changed mid-episode is used from the next step on
            rm.AGV_MOVE_PENALTY = -0.77
        if t == 250:   # a replaced reward_calculator object too
            sim.reward_calculator = rm = type(rm)(ORDER_COMPLETE_REWARD=55.5, AGV_DELIVERY_REWARD=3.25)
        acts = O.actions(4, 1, t, None)
        actions = {a: int(acts[i]) for i, a in enumerate(spec.AGENTS)}
        obs, rew, term, trunc, info = sim.step(actions)
        oc = info["agv"]["orders_completed"]
        pk = info["agv"]["total_products_packaged"]
        g = rm.calculate_global_reward(oc - prev_orders, pk - prev_pk, 10)
        local = {a: rm.calculate_local_reward(a, actions[a], info[a]["action_result"]) for a in spec.AGENTS}
        exp = rm.combine_rewards(g, local, 8)
        for a in spec.AGENTS:
            assert rew[a] == exp[a], (t, a, rew[a], exp[a])
        prev_orders, prev_pk = oc, pk
        if term["agv"] or trunc["agv"]:
            sim.reset(num_orders=3)
            prev_orders = prev_pk = 0


def test_transition_memory_dropin_matches_golden(M):
    d = np.load(f"{P.GOLDEN}/gae.npz")
    agents = M["spec"].AGENTS
    for c in range(3):
        g, l = d[f"c{c}_gamma_lamb"]
        rw, v, boots, se = d[f"c{c}_rewards"], d[f"c{c}_values"], d[f"c{c}_boots"], d[f"c{c}_seg_end"]
        mem = M["TM"].MultiAgentTransitionMemory(agents, float(g), float(l), True)
        start = 0
        for si, end in enumerate(np.nonzero(se)[0] + 1):
            for t in range(start, end):
                mem.put({a: None for a in agents}, {a: 0 for a in agents},
                        {a: float(rw[t, i]) for i, a in enumerate(agents)}, {a: None for a in agents},
                        {a: torch.tensor(v[t, i]) for i, a in enumerate(agents)})
            mem.finish_trajectory({a: float(boots[si, i]) for i, a in enumerate(agents)})
            start = end
        ret = np.array([mem.return_lst[a] for a in agents]).T
        adv = np.array([mem.adv_lst[a] for a in agents]).T
        assert P.bits_equal(ret, d[f"c{c}_returns"]), c
        assert P.bits_equal(adv, d[f"c{c}_adv"]), c


def test_state_render_spaces(M):
    env = M["W"].FJSPParallelEnv(render_mode="rgb_array")
    env.reset(seed=0)
    st = env.state()
    # np.concatenate promotes int32 + float32 to float64, as in the reference (wrapper :119-136)
    assert st.dtype == np.float64 and st.shape == (38 + 29 + 4,)
    grid = env.render()
    assert grid.shape == (4, 6, 3) and tuple(grid[0, 0]) == (0, 0, 0)
    assert env.action_space("agv").n == 8 and env.action_space("packaging_red").n == 3
    sp = env.observation_space("agv")
    assert list(sp.spaces.keys()) == sorted(REF_KEYS["agv"])
    assert env.unwrapped is env
