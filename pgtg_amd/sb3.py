"""Stable-Baselines3-style vector env over the device batch (replaces the `SubprocVecEnv` of
pgtg/train.py:54-55).

`PGTGSB3VecEnv(num_envs, max_episode_steps=100, **PGTGEnv kwargs)` follows SB3's `VecEnv` protocol
(duck-typed, stable_baselines3 need not be installed): `reset() -> obs`, `step_async(actions)` /
`step_wait() -> (obs, rewards, dones, infos)` with `infos[i]["terminal_observation"]` and
`infos[i]["TimeLimit.truncated"]` for finished envs.  Observations are the `FlattenObservation`
vectors of pgtg/train.py:40 (pgtg_amd/flat.py), as float32 numpy arrays because SB3 policies take
host arrays; `max_episode_steps` is the `TimeLimit(100)` wrapper of pgtg/train.py:39, applied
in-kernel (truncation and auto-reset in the same step).
"""
from __future__ import annotations

from typing import Any

import numpy as np

from .flat import flat_dim, flatten_obs
from .vector import PGTGVecEnv


class PGTGSB3VecEnv:
    def __init__(self, num_envs: int, map_path: str | None = None, *, max_episode_steps: int | None = 100,
                 device: int | None = None, seed: int = 0, **kwargs: Any):
        self.venv = PGTGVecEnv(num_envs, map_path, device=device, autoreset=True,
                               max_episode_steps=max_episode_steps, **kwargs)
        self.spec = self.venv.spec
        self.num_envs = num_envs
        self.obs_dim = flat_dim(self.spec)
        self._seed = seed
        self._actions = None
        try:
            from gymnasium import spaces
            self.observation_space = spaces.Box(low=-99, high=99, shape=(self.obs_dim,), dtype=np.float32)
            self.action_space = spaces.Discrete(9)
        except ImportError:
            self.observation_space = None
            self.action_space = None

    # -- VecEnv protocol ------------------------------------------------------------------------
    def seed(self, seed: int | None = None):
        self._seed = 0 if seed is None else int(seed)
        return [self._seed + i for i in range(self.num_envs)]

    def reset(self) -> np.ndarray:
        obs, _ = self.venv.reset(seed=self._seed)
        return flatten_obs(self.spec, obs).cpu().numpy()

    def step_async(self, actions) -> None:
        a = np.asarray(actions).reshape(self.num_envs)
        if a.size and (a.min() < 0 or a.max() > 8):  # an out-of-space action raises (environment.py:1118)
            raise KeyError(int(a[(a < 0) | (a > 8)][0]))
        self._actions = a.astype(np.uint8)

    def step_wait(self):
        import torch
        obs, reward, term, trunc, infos = self.venv.step(torch.as_tensor(self._actions))
        flat = flatten_obs(self.spec, obs).cpu().numpy()
        rew = reward.to(torch.float32).cpu().numpy()
        term_h, trunc_h = term.cpu().numpy().astype(bool), trunc.cpu().numpy().astype(bool)
        dones = term_h | trunc_h
        out_infos: list[dict[str, Any]] = [{} for _ in range(self.num_envs)]
        if dones.any():
            final = flatten_obs(self.spec, infos["final_observation"]).cpu().numpy()
            for i in np.nonzero(dones)[0]:
                out_infos[i]["terminal_observation"] = final[i]
                out_infos[i]["TimeLimit.truncated"] = bool(trunc_h[i] and not term_h[i])
        if "cost" in infos:
            cost = infos["cost"].cpu().numpy()
            for i in range(self.num_envs):
                out_infos[i]["cost"] = float(cost[i])
        return flat, rew, dones, out_infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self) -> None:
        self.venv.close()

    def get_attr(self, name: str, indices=None):
        n = self.num_envs if indices is None else len(list(indices))
        return [getattr(self.spec, name, None)] * n

    def set_attr(self, name: str, value, indices=None) -> None:
        raise AttributeError("the device batch has no per-env Python attributes")

    def env_method(self, name: str, *args, indices=None, **kwargs):
        raise AttributeError("the device batch has no per-env Python methods")

    def env_is_wrapped(self, wrapper_class, indices=None):
        n = self.num_envs if indices is None else len(list(indices))
        return [False] * n
