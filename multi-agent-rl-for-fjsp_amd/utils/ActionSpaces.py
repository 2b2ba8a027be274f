"""ActionSpaces API mirror (reference: utils/ActionSpaces.py): Discrete(n) per agent type."""
from .. import spaces
from ..spec import ACTION_NAMES


def _discrete(agent):
    return lambda: spaces.Discrete(len(ACTION_NAMES[agent]) if agent == "agv" else 3)


class ActionSpaces:
    pickup_station = staticmethod(_discrete("pickup_station"))
    agv = staticmethod(_discrete("agv"))
    small_machine = staticmethod(_discrete("small_machine"))
    big_machine = staticmethod(_discrete("big_machine"))
    packaging = staticmethod(_discrete("packaging_blue_1"))
