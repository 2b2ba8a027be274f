"""Makes the fjsp_amd package importable for the reference-named shim modules in this folder.

Put this folder (multi-agent-rl-for-fjsp_amd/dropin) first on sys.path and the reference's own
train.py / a2c.py import the GPU environment instead of the SimPy one."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if REPO not in sys.path:
    sys.path.append(REPO)


def load(name):
    return importlib.import_module("multi-agent-rl-for-fjsp_amd." + name)
