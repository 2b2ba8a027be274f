"""Observation / action layout shared by the kernels and the Python facade.

Field order = the reference's observation dict insertion order per agent
(PickupStationAgent.py:131-140, AGVAgent.py:60-75, MachineAgent.py:64-69,
PackagingAgent.py:266-271), split by dtype into the SoA blocks of include/fjsp.h.
"""
import numpy as np

AGENTS = ["pickup_station", "agv", "small_machine", "big_machine",
          "packaging_blue_1", "packaging_blue_2", "packaging_red", "packaging_green"]
N_ACTIONS = [3, 8, 3, 3, 3, 3, 3, 3]
MASK_OFFSETS = [0, 3, 11, 14, 17, 20, 23, 26]

PICKUP_FIELDS = ["order_size", "products_remaining", "next_product_type", "next_product_color",
                 "current_tray_type", "current_tray_color", "current_tray_count"]
AGV_FIELDS = ["position", "carrying_tray", "tray_product_count", "tray_type", "tray_needs_processing",
              "tray_needs_packaging", "pickup_ready_trays", "small_machine_busy", "big_machine_busy",
              "small_machine_ready", "big_machine_ready", "storage_tray_count"]
STATION_FIELDS = ["is_busy", "processing_progress", "queue_length"]

# agent -> action names (FJSPSimulation.py:339-348)
ACTION_NAMES = {
    "pickup_station": ["IDLE", "LOAD_PRODUCT", "SIGNAL_READY"],
    "agv": ["IDLE", "TO_PICKUP", "TO_SMALL_M", "TO_BIG_M", "TO_STORAGE", "TO_PACKAGING", "PICKUP", "DROP"],
    "small_machine": ["IDLE", "START_PROC", "SIGNAL_DONE"],
    "big_machine": ["IDLE", "START_PROC", "SIGNAL_DONE"],
    "packaging_blue_1": ["IDLE", "START_PKG"],
    "packaging_blue_2": ["IDLE", "START_PKG"],
    "packaging_red": ["IDLE", "START_PKG"],
    "packaging_green": ["IDLE", "START_PKG"],
}

# action-result words -> reference result dict keys (bit i = key i; bit 7 = executed)
RESULT_KEYS = {
    "pickup_station": ["success", "product_loaded", "tray_completed", "idle_with_orders"],
    "agv": ["success", "invalid_action", "moved", "pickup_success", "drop_success", "delivered_to_packaging"],
    "machine": ["success", "started_processing", "completed_processing", "idle_with_queue"],
    "packaging": ["success", "started_packaging", "completed_packaging", "idle_with_queue"],
}
RESULT_INT = {"agv": "distance", "packaging": "products_completed_this_step"}


def agent_kind(a):
    if a in ("small_machine", "big_machine"):
        return "machine"
    if a.startswith("packaging"):
        return "packaging"
    return a


def decode_result(agent, action, word):
    """Rebuild the reference's action-result dict (e.g. MachineAgent.py:106-112)."""
    word = int(word)
    if not word & 0x80:
        return {}
    kind = agent_kind(agent)
    d = {"action": int(action)}
    keys = RESULT_KEYS[kind]
    if kind == "pickup_station":
        order = ["success", "product_loaded", "tray_completed", "idle_with_orders"]
    elif kind == "agv":
        order = ["success", "invalid_action", "moved", "distance", "pickup_success", "drop_success",
                 "delivered_to_packaging"]
    elif kind == "machine":
        order = ["success", "started_processing", "completed_processing", "idle_with_queue"]
    else:
        order = ["success", "started_packaging", "completed_packaging", "idle_with_queue",
                 "products_completed_this_step"]
    for k in order:
        if k in keys:
            d[k] = bool(word >> keys.index(k) & 1)
        else:
            d[k] = (word >> 16) & 0xFFFF
    return d


_I32, _I8, _F32 = np.dtype(np.int32), np.dtype(np.int8), np.dtype(np.float32)


def obs_dicts(i32, i8, f32, mask):
    """One env's SoA observation columns -> the reference's dict of numpy arrays (fresh arrays:
    the values are taken as Python numbers once, each agent's action mask is its own slice of
    one fresh copy of the 29 mask bytes)."""
    a, b, c, m = i32.tolist(), i8.tolist(), f32.tolist(), np.array(mask, dtype=_I8)
    arr = np.array
    obs = {}
    p = {k: arr(a[i], _I32) for i, k in enumerate(PICKUP_FIELDS)}
    p["action_mask"] = m[0:3]
    obs["pickup_station"] = p
    g = {"position": arr(a[7:9], _I32)}
    for j, k in enumerate(AGV_FIELDS[1:]):
        g[k] = arr(a[9 + j], _I32)
    g["action_mask"] = m[3:11]
    obs["agv"] = g
    for s, name in enumerate(AGENTS[2:]):
        obs[name] = {"is_busy": arr(b[2 * s], _I8), "processing_progress": arr(c[s], _F32),
                     "queue_length": arr(b[2 * s + 1], _I8), "action_mask": m[11 + 3 * s: 14 + 3 * s]}
    return obs


# a2c flat layout: per agent sorted keys without action_mask (a2c.py:137-151)
def a2c_feature_index():
    """Indices into the concatenation [i32(20) | i8(12) | f32(6)] producing a2c's global state
    (dim 38, agent order, sorted keys per agent; a2c.py:153-166)."""
    idx = []
    names = {}
    for i, k in enumerate(PICKUP_FIELDS):
        names[("pickup_station", k)] = [i]
    names[("agv", "position")] = [7, 8]
    for j, k in enumerate(AGV_FIELDS[1:]):
        names[("agv", k)] = [9 + j]
    for s, name in enumerate(AGENTS[2:]):
        names[(name, "is_busy")] = [20 + 2 * s]
        names[(name, "queue_length")] = [20 + 2 * s + 1]
        names[(name, "processing_progress")] = [32 + s]
    for a in AGENTS:
        keys = sorted(k for (ag, k) in names if ag == a)
        for k in keys:
            idx.extend(names[(a, k)])
    return idx


A2C_OBS_DIMS = {"pickup_station": 7, "agv": 13, "small_machine": 3, "big_machine": 3,
                "packaging_blue_1": 3, "packaging_blue_2": 3, "packaging_red": 3, "packaging_green": 3}
