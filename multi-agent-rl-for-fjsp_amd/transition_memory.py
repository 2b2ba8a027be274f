"""MultiAgentTransitionMemory drop-in (reference: transition_memory.py:6-133).

Same per-agent list API (put / finish_trajectory / get / clear / has_data); the return and GAE
scans of finish_trajectory (transition_memory.py:83-105) run in the fp64 HIP kernel k_gae
(fjsp_gae), one lane per agent column, with Python's unfused operation order.
"""
import numpy as np
import torch

from .vec_env import gae as _gae


class MultiAgentTransitionMemory:
    def __init__(self, agent_ids, gamma, lamb, use_gae=True, device=None):
        self.agent_ids = agent_ids
        self.gamma = gamma
        self.lamb = lamb
        self.use_gae = use_gae
        if not torch.cuda.is_available():
            raise RuntimeError("MultiAgentTransitionMemory (fjsp_amd) computes GAE with the HIP kernel; no GPU visible")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.clear()

    def put(self, observations, actions, rewards, logprobs, values):
        for a in self.agent_ids:
            if a in observations:
                self.obs_lst[a].append(observations[a])
                self.action_lst[a].append(actions[a])
                self.reward_lst[a].append(rewards[a])
                self.logprob_lst[a].append(logprobs[a])
                self.value_lst[a].append(values[a])

    @staticmethod
    def _scalar(v):
        return v.detach().item() if torch.is_tensor(v) else float(v)

    def finish_trajectory(self, next_values):
        # gather every agent's pending segment; agents with equal lengths share one launch
        segs = {}
        for a in self.agent_ids:
            start = self.traj_start[a]
            r = self.reward_lst[a][start:]
            if len(r) == 0:
                continue
            v = [self._scalar(x) for x in self.value_lst[a][start:]]
            segs.setdefault(len(r), []).append((a, r, v, float(next_values.get(a, 0.0))))
        for T, group in segs.items():
            M = len(group)
            rw = torch.tensor(np.array([g[1] for g in group], dtype=np.float64).T.copy(), device=self.device)
            vv = torch.tensor(np.array([g[2] for g in group], dtype=np.float64).T.copy(), device=self.device)
            boot = torch.tensor([g[3] for g in group], dtype=torch.float64, device=self.device)
            done = torch.zeros(T, M, dtype=torch.uint8, device=self.device)
            ret, adv = _gae(rw, vv, done, boot, self.gamma, self.lamb)
            ret = ret.cpu().numpy()
            adv = adv.cpu().numpy()
            for j, (a, r, v, nv) in enumerate(group):
                self.return_lst[a].extend(ret[:, j].tolist())
                if self.use_gae:
                    self.adv_lst[a].extend(adv[:, j].tolist())
                else:   # _compute_advantages: A = R - V (transition_memory.py:92-94)
                    self.adv_lst[a].extend((ret[:, j] - np.asarray(v)).tolist())
                self.traj_start[a] = len(self.reward_lst[a])

    def get(self, agent_id):
        return (self.obs_lst[agent_id], self.action_lst[agent_id], self.reward_lst[agent_id],
                self.logprob_lst[agent_id], self.return_lst[agent_id], self.value_lst[agent_id],
                self.adv_lst[agent_id])

    def clear(self):
        for name in ("obs_lst", "action_lst", "reward_lst", "logprob_lst", "value_lst", "return_lst", "adv_lst"):
            setattr(self, name, {a: [] for a in self.agent_ids})
        self.traj_start = {a: 0 for a in self.agent_ids}

    def has_data(self):
        return any(len(self.obs_lst[a]) > 0 for a in self.agent_ids)
