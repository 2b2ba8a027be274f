"""RewardModel API mirror (reference: utils/RewardModel.py:7-110).

The rewards of every step are computed inside the HIP step kernel from these weights (passed
through fjsp_set_reward_weights); this class keeps the reference's tunable dataclass surface so
callers can read or change the weights.  ``weights()`` is the fp64 vector the kernel consumes.
The calculate_* methods restate the formulas for callers that use them directly.
"""
from dataclasses import dataclass, fields

from ..spec import agent_kind


@dataclass
class RewardModel:
    ORDER_COMPLETE_REWARD: float = 100.0
    THROUGHPUT_BONUS: float = 10.0
    TIME_PENALTY: float = -0.1
    PICKUP_LOAD_REWARD: float = 1.0
    PICKUP_TRAY_COMPLETE: float = 5.0
    PICKUP_IDLE_PENALTY: float = -1.0
    AGV_DELIVERY_REWARD: float = 2.0
    AGV_MOVE_PENALTY: float = -0.1
    AGV_PACKAGING_DELIVERY: float = 10.0
    AGV_INVALID_ACTION: float = -5.0
    MACHINE_COMPLETE_REWARD: float = 5.0
    MACHINE_START_REWARD: float = 1.0
    MACHINE_IDLE_PENALTY: float = -2.0
    PACKAGING_COMPLETE_REWARD: float = 20.0
    PACKAGING_START_REWARD: float = 2.0
    PACKAGING_IDLE_PENALTY: float = -1.0

    def weights(self):
        """Weights in fjsp_reward_weights order (include/fjsp.h)."""
        return tuple(float(getattr(self, n)) for n in _WEIGHT_NAMES)

    # (weight, result key, only-when-action-0) terms per agent kind, in the reference's order
    _TERMS = {
        "pickup_station": (("PICKUP_LOAD_REWARD", "product_loaded", False),
                           ("PICKUP_TRAY_COMPLETE", "tray_completed", False),
                           ("PICKUP_IDLE_PENALTY", "idle_with_orders", True)),
        "agv": (("AGV_DELIVERY_REWARD", "pickup_success", False), ("AGV_DELIVERY_REWARD", "drop_success", False),
                ("AGV_PACKAGING_DELIVERY", "delivered_to_packaging", False), ("AGV_MOVE_PENALTY", "moved", False),
                ("AGV_INVALID_ACTION", "invalid_action", False)),
        "machine": (("MACHINE_START_REWARD", "started_processing", False),
                    ("MACHINE_COMPLETE_REWARD", "completed_processing", False),
                    ("MACHINE_IDLE_PENALTY", "idle_with_queue", True)),
        "packaging": (("PACKAGING_START_REWARD", "started_packaging", False),
                      ("PACKAGING_COMPLETE_REWARD", "completed_packaging", False),
                      ("PACKAGING_IDLE_PENALTY", "idle_with_queue", True)),
    }

    def calculate_global_reward(self, orders_completed, products_packaged, time_elapsed):
        reward = self.ORDER_COMPLETE_REWARD * orders_completed
        reward += self.THROUGHPUT_BONUS * products_packaged
        reward += self.TIME_PENALTY * time_elapsed
        return reward

    def calculate_local_reward(self, agent, action_taken, action_result):
        """``agent``: an agent id (e.g. 'small_machine') or a reference AgentType-like with a name."""
        name = agent if isinstance(agent, str) else getattr(agent, "name", str(agent)).lower()
        kind = {"pickup_station": "pickup_station", "agv": "agv", "small_machine": "machine",
                "big_machine": "machine", "packaging": "packaging"}.get(name, agent_kind(name))
        reward = 0.0
        for wname, key, idle in self._TERMS[kind]:
            if action_result.get(key, False) and (not idle or action_taken == 0):
                reward += getattr(self, wname)
        return reward

    def combine_rewards(self, global_reward, local_rewards, num_agents):
        return {a: global_reward / num_agents + r for a, r in local_rewards.items()}


_WEIGHT_NAMES = tuple(f.name for f in fields(RewardModel))   # dataclass field order = fjsp_reward_weights order
