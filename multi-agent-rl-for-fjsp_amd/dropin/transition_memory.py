"""Shim: `from transition_memory import MultiAgentTransitionMemory` -> GAE on the GPU."""
from _bootstrap import load

MultiAgentTransitionMemory = load("transition_memory").MultiAgentTransitionMemory
