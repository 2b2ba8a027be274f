"""FJSPParallelEnv drop-in (reference: FJSPParallelEnvWrapper.py:9-137).

PettingZoo Parallel API over the GPU-stepped FJSPSimulation facade: possible_agents / agents,
observation_space / action_space, reset(seed, options={'num_orders': k}), step(actions) that
drops every agent once the episode terminates or truncates, state(), render(), close(),
unwrapped.  Inherits pettingzoo.ParallelEnv when pettingzoo is installed.
"""
import numpy as np

from .FJSPSimulation import LOCATION_POSITIONS, FJSPSimulation

try:  # pragma: no cover - depends on the environment
    from pettingzoo import ParallelEnv as _Base
except ImportError:
    class _Base:
        @property
        def unwrapped(self):
            return self

        @property
        def num_agents(self):
            return len(self.agents)

        @property
        def max_num_agents(self):
            return len(self.possible_agents)


class FJSPParallelEnv(_Base):
    metadata = {"name": "fjsp_v1", "render_modes": ["human", "rgb_array"], "is_parallelizable": True}

    def __init__(self, config=None, render_mode=None, device=None):
        self.simulation = FJSPSimulation(config, device=device)
        self.render_mode = render_mode
        self.possible_agents = self.simulation.get_agent_ids()
        self.agents = self.possible_agents.copy()

    def observation_space(self, agent):
        return self.simulation.observation_space(agent)

    def action_space(self, agent):
        return self.simulation.action_space(agent)

    def reset(self, seed=None, options=None):
        self.agents = self.possible_agents.copy()
        num_orders = options.get("num_orders") if options else None
        return self.simulation.reset(seed, num_orders=num_orders)

    def step(self, actions):
        obs, rewards, terms, truncs, infos = self.simulation.step(actions)
        if True in terms.values() or True in truncs.values():   # (the filter is a no-op otherwise)
            self.agents = [a for a in self.agents if not terms.get(a, False) and not truncs.get(a, False)]
        return obs, rewards, terms, truncs, infos

    def state(self):
        """Global state (FJSPParallelEnvWrapper.py:119-136): every agent's obs in sorted-key
        order (action masks included) + [len(orders), completed, packaged, now] as float32."""
        obs = self.simulation.get_observations()
        parts = []
        for a in self.possible_agents:
            for k in sorted(obs[a].keys()):
                parts.append(np.asarray(obs[a][k]).flatten())
        prog = self.simulation._view()
        parts.append(np.array([self.simulation.orders_count, prog.orders_completed, prog.total_packaged,
                               self.simulation.sim_time], dtype=np.float32))
        return np.concatenate(parts)

    def render(self):
        if self.render_mode == "human":
            v = self.simulation._view()
            print(f"Step {self.simulation.current_step} | SimTime: {self.simulation.sim_time} | "
                  f"Orders: {v.orders_completed}/{v.num_orders} | Packaged: {v.total_packaged} | "
                  f"AGV at ({v.agv_row}, {v.agv_col}) carrying={'Yes' if v.agv_carrying else 'No'}")
            return None
        if self.render_mode == "rgb_array":
            grid = np.ones((4, 6, 3), dtype=np.uint8) * 255
            colors = {"PICKUP": [0, 255, 0], "SMALL_MACHINE": [0, 0, 255], "BIG_MACHINE": [255, 0, 0],
                      "STORAGE": [128, 128, 128], "PACKAGING": [255, 255, 0]}
            for loc, (r, c) in LOCATION_POSITIONS.items():
                grid[r, c] = colors[loc]
            r, c = self.simulation.agv.position
            grid[r, c] = [0, 0, 0]
            return grid
        return None

    def close(self):
        pass
