"""MI355X-native vectorised FJSP environment (drop-in for FARIDKH/Multi-agent-RL-for-FJSP's
FJSPSimulation / FJSPParallelEnv hot path and its GAE/return scan).

The package directory name is not a Python identifier; import it with
``importlib.import_module("multi-agent-rl-for-fjsp_amd")`` or put this directory itself on
``sys.path`` to use the reference-named drop-in modules (``FJSPParallelEnvWrapper``,
``FJSPSimulation``, ``transition_memory``).
"""
from . import _native  # noqa: F401
from .spec import AGENTS, N_ACTIONS  # noqa: F401


def build(force=False):
    return _native.build(force=force)


def __getattr__(name):
    # lazy: importing the package must not require a GPU
    if name in ("FJSPVecEnv", "Buffers", "gae"):
        from . import vec_env
        return getattr(vec_env, name)
    raise AttributeError(name)
