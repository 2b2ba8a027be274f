"""Stand-in for ``gymnasium`` (TEST INFRASTRUCTURE, used only to import the reference here).

The reference only declares spaces (utils/ObservationSpaces.py, utils/ActionSpaces.py) and
reads ``.n`` / ``.shape`` / ``.spaces`` (a2c.py:118-135); ``sample()`` is used only by the
never-called ``train.test_environment`` (train.py:268).
"""
from . import spaces  # noqa: F401

Env = object
