"""Shim: `from FJSPParallelEnvWrapper import FJSPParallelEnv` -> the GPU environment."""
from _bootstrap import load

FJSPParallelEnv = load("FJSPParallelEnvWrapper").FJSPParallelEnv
