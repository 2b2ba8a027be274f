"""The drop-in facade's host helper (csrc/fjsp_facade.c, `_facade.obs_dicts`) against its Python
definition (spec.obs_dicts) and the reference's own observation records (no GPU: the helper only
turns one env's record columns into the reference's dicts).

Every record of tests/golden/traces.npz (observations of the reference's FJSPParallelEnv,
flattened by gen_golden.flatten_obs) is rebuilt into dicts by the C helper and flattened again:
byte-equal, with the reference's structure (PickupStationAgent.py:87-96, AGVAgent.py:60-75,
MachineAgent.py:64-69, PackagingAgent.py:266-271): agent order, key order, 0-d arrays of the
field dtype, the AGV's position a 2-vector, int8 action masks of each agent's action count."""
import importlib
import os

import numpy as np
import pytest

from tests import gpu_util as G
from tests.golden.gen_golden import flatten_obs

S = importlib.import_module("multi-agent-rl-for-fjsp_amd.spec")


@pytest.fixture(scope="module")
def F():
    return G.native.facade()


def _same(a, b):
    assert list(a) == list(b)
    for ag in a:
        assert list(a[ag]) == list(b[ag]), ag
        for k in a[ag]:
            x, y = a[ag][k], b[ag][k]
            assert type(x) is type(y) is np.ndarray, (ag, k)
            assert x.dtype == y.dtype and x.shape == y.shape and x.tobytes() == y.tobytes(), (ag, k)


def test_obs_dicts_c_round_trips_reference_records(F):
    d = np.load(os.path.join(G.REPO, "tests", "golden", "traces.npz"))
    names = sorted({k[: -len("_obs_i32")] for k in d.files if k.endswith("_obs_i32")})
    assert names
    n = 0
    for name in names:
        i32, i8, f32, m = (d[f"{name}_{f}"] for f in ("obs_i32", "obs_i8", "obs_f32", "masks"))
        for t in range(0, i32.shape[0], 7):
            obs = F.obs_dicts(i32[t], i8[t], f32[t], m[t])
            back = flatten_obs(obs)
            assert all(x.tobytes() == y.tobytes() for x, y in zip(back, (i32[t], i8[t], f32[t], m[t]))), (name, t)
            _same(obs, S.obs_dicts(i32[t], i8[t], f32[t], m[t]))
            n += 1
    assert n > 500


def test_obs_dicts_c_structure(F):
    rng = np.random.default_rng(1)
    i32 = rng.integers(-5, 100, 20).astype(np.int32)
    i8 = rng.integers(-3, 50, 12).astype(np.int8)
    f32 = rng.random(6).astype(np.float32)
    m = rng.integers(0, 2, 29).astype(np.int8)
    obs = F.obs_dicts(i32, i8, f32, m)
    assert list(obs) == S.AGENTS
    assert list(obs["pickup_station"]) == S.PICKUP_FIELDS + ["action_mask"]
    assert list(obs["agv"]) == S.AGV_FIELDS + ["action_mask"]
    assert obs["agv"]["position"].shape == (2,) and obs["agv"]["position"].tolist() == i32[7:9].tolist()
    for a, na, off in zip(S.AGENTS, S.N_ACTIONS, S.MASK_OFFSETS):
        mk = obs[a]["action_mask"]
        assert mk.dtype == np.int8 and mk.shape == (na,) and mk.tolist() == m[off:off + na].tolist()
    for s, a in enumerate(S.AGENTS[2:]):
        o = obs[a]
        assert list(o) == S.STATION_FIELDS + ["action_mask"]
        assert o["is_busy"].shape == () and o["is_busy"].dtype == np.int8 and int(o["is_busy"]) == i8[2 * s]
        assert o["processing_progress"].dtype == np.float32 and float(o["processing_progress"]) == f32[s]
        assert o["queue_length"].dtype == np.int8 and int(o["queue_length"]) == i8[2 * s + 1]
    # fresh arrays: the next call's values never show through an earlier result
    i32[0] += 1
    again = F.obs_dicts(i32, i8, f32, m)
    assert int(again["pickup_station"]["order_size"]) == int(obs["pickup_station"]["order_size"]) + 1


def test_obs_dicts_c_rejects_short_buffers(F):
    z = np.zeros(40, np.int32)
    with pytest.raises(ValueError):
        F.obs_dicts(z[:19], np.zeros(12, np.int8), np.zeros(6, np.float32), np.zeros(29, np.int8))
    with pytest.raises(ValueError):
        F.obs_dicts(z, np.zeros(12, np.int8), np.zeros(6, np.float32), np.zeros(28, np.int8))
