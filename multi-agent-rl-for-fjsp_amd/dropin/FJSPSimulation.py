"""Shim: `from FJSPSimulation import FJSPSimulation` -> the GPU environment (N = 1)."""
from _bootstrap import load

_m = load("FJSPSimulation")
FJSPSimulation = _m.FJSPSimulation
CONFIG = _m.CONFIG
