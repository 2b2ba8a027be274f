"""ObservationSpaces API mirror (reference: utils/ObservationSpaces.py).

Built from a table: (key, kind, arg) per agent type; the values are the reference's
declared space sizes (its spaces only size networks, a2c.py:118-135)."""
import numpy as np

from .. import spaces

_GRID = (4, 6)        # CONFIG grid_rows / grid_cols
_TRAY_CAP = 5         # CONFIG tray_capacity

_TABLE = {
    "pickup_station": [("order_size", "d", 21), ("products_remaining", "d", 21), ("next_product_type", "d", 4),
                       ("next_product_color", "d", 4), ("current_tray_type", "d", 4),
                       ("current_tray_color", "d", 4), ("current_tray_count", "d", 6), ("action_mask", "m", 3)],
    "agv": [("position", "md", _GRID), ("carrying_tray", "d", 2), ("tray_product_count", "d", _TRAY_CAP + 1),
            ("tray_type", "d", 4), ("tray_needs_processing", "d", 2), ("tray_needs_packaging", "d", 2),
            ("pickup_ready_trays", "d", 10), ("small_machine_busy", "d", 2), ("big_machine_busy", "d", 2),
            ("small_machine_ready", "d", 10), ("big_machine_ready", "d", 10), ("storage_tray_count", "d", 100),
            ("action_mask", "m", 8)],
    "machine": [("is_busy", "d", 2), ("processing_progress", "b", 1), ("queue_length", "d", 10),
                ("action_mask", "m", 3)],
    "packaging": [("is_busy", "d", 2), ("processing_progress", "b", 1), ("queue_length", "d", 20),
                  ("action_mask", "m", 3)],
}


def _build(kind):
    d = {}
    for key, t, arg in _TABLE[kind]:
        if t == "d":
            d[key] = spaces.Discrete(arg)
        elif t == "md":
            d[key] = spaces.MultiDiscrete(list(arg))
        elif t == "b":
            d[key] = spaces.Box(low=0, high=1, shape=(arg,), dtype=np.float32)
        else:
            d[key] = spaces.Box(low=0, high=1, shape=(arg,), dtype=np.int8)
    return spaces.Dict(d)


class ObservationSpaces:
    @staticmethod
    def pickup_station():
        return _build("pickup_station")

    @staticmethod
    def agv():
        return _build("agv")

    @staticmethod
    def small_machine():
        return _build("machine")

    @staticmethod
    def big_machine():
        return _build("machine")

    @staticmethod
    def packaging(color=None):
        return _build("packaging")
