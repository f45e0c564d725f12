"""Stable-Baselines3-style vector env over the device batch (replaces the `SubprocVecEnv` of
pgtg/train.py:54-55).

`PGTGSB3VecEnv(num_envs, max_episode_steps=100, **PGTGEnv kwargs)` follows SB3's `VecEnv` protocol
(duck-typed, stable_baselines3 need not be installed): `reset() -> obs`, `step_async(actions)` /
`step_wait() -> (obs, rewards, dones, infos)` with `infos[i]["terminal_observation"]` and
`infos[i]["TimeLimit.truncated"]` for finished envs (`infos` a lazy sequence, `VecInfos`: no per-env
Python loop in the step).  Observations are the `FlattenObservation`
vectors of pgtg/train.py:40 (pgtg_amd/flat.py), as float32 numpy arrays because SB3 policies take
host arrays (views of page-locked buffers that are fresh for every step, so a caller may keep them like
SubprocVecEnv's arrays; `zero_copy=True` reuses two buffer sets in turn, a step's arrays then being valid
until the step after next); `max_episode_steps` is the `TimeLimit(100)` wrapper of pgtg/train.py:39,
applied in-kernel (truncation and auto-reset in the same step).

`device_obs=True` keeps everything on the env's GPU for device-side rollout buffers and policies:
observations, rewards and dones come back as torch tensors (`obs_dtype`: float32 by default; int8 is
exact as well, every flattened value being a 0/1 one-hot entry or a velocity in Box(-99, 99)),
actions may be a device tensor, and the infos (`DeviceVecInfos`)
carry the batch's terminal observations as one [N, D] tensor (valid on the rows of finished envs),
converted to SB3's per-env dicts only if an entry is read.  Nothing crosses PCIe in the step.  The
flattened rows (float32 / int8) are written by the HIP kernel k_flatten inside the step (include/pgtg.h
pgtg_set_flat_outputs) into tensors that are fresh for every step; other dtypes go through flatten_obs.
"""
from __future__ import annotations

from collections.abc import Sequence
from typing import Any

import numpy as np

from .flat import flat_dim, flatten_obs
from .vector import PGTGVecEnv


class VecInfos(Sequence):
    """SB3's per-env `infos` list without per-env Python work in the step: the batch's arrays are kept
    and env i's dict ({"terminal_observation", "TimeLimit.truncated"} when it finished, "cost" with
    separate_reward_cost) is built when it is first read and kept, so a step costs O(1) host work
    whatever the batch size; callers that read every entry pay for what they read (SB3's VecMonitor,
    which pgtg/train.py:55 wraps around the env, reads them all: `list(infos[:])` per step)."""

    def __init__(self, dones, truncated, final, cost, final_rows=None):
        """final: the terminal observations, one row per env ([N, D]), or with `final_rows` one row per
        finished env in env order (final_rows[i] = env i's row)."""
        self._dones, self._trunc, self._final, self._cost = dones, truncated, final, cost
        self._rows = final_rows
        # env i's dict, built on its first read and returned on every later one: SB3 wrappers
        # (VecNormalize, VecFrameStack, VecTransposeImage) rewrite infos[i]["terminal_observation"] in
        # place and rely on reading their own value back, as from SubprocVecEnv's list
        self._cache: dict[int, dict[str, Any]] = {}
        self._all: list | None = None

    def __len__(self) -> int:
        return len(self._dones)

    def _make(self, i: int) -> dict[str, Any]:
        d: dict[str, Any] = {}
        if self._dones[i]:
            d["terminal_observation"] = self._final[i if self._rows is None else int(self._rows[i])]
            d["TimeLimit.truncated"] = bool(self._trunc[i])
        if self._cost is not None:
            d["cost"] = float(self._cost[i])
        return d

    def _materialize(self) -> list:
        """Every entry at once (VecMonitor's list(infos[:])): plain dicts, then the finished envs'."""
        if self._all is None:
            n = len(self)
            if self._cost is None:
                lst = [{} for _ in range(n)]
            else:
                lst = [{"cost": c} for c in self._cost.tolist()]
            for i in np.nonzero(self._dones)[0].tolist():
                lst[i].update(self._make(i))
            for i, d in self._cache.items():  # entries already handed out stay the same objects
                lst[i] = d
            self._all = lst
        return self._all

    def __getitem__(self, i):
        if isinstance(i, slice):
            return self._materialize()[i]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        if self._all is not None:
            return self._all[i]
        d = self._cache.get(i)
        if d is None:
            d = self._cache[i] = self._make(i)
        return d

    def finished(self) -> np.ndarray:
        """Indices of the envs whose episode ended this step (vectorised access)."""
        return np.nonzero(self._dones)[0]


class DeviceVecInfos(Sequence):
    """The infos of a `device_obs` step: the batch's tensors on the device (`dones`, `truncated`,
    `terminal_observation` [N, D] with valid rows where done, `cost`), and SB3's per-env dicts on
    demand (the first per-env read copies the masks to the host once)."""

    def __init__(self, dones, truncated, final, cost):
        self.dones, self.truncated, self.terminal_observation, self.cost = dones, truncated, final, cost
        self._host: VecInfos | None = None

    def _h(self) -> VecInfos:
        if self._host is None:
            d = self.dones.cpu().numpy()
            self._host = VecInfos(d, self.truncated.cpu().numpy(), self.terminal_observation,
                                  None if self.cost is None else self.cost.cpu().numpy())
        return self._host

    def __len__(self) -> int:
        return int(self.dones.shape[0])

    def __getitem__(self, i):
        return self._h()[i]

    def finished(self):
        return self._h().finished()


class PGTGSB3VecEnv:
    def __init__(self, num_envs: int, map_path: str | None = None, *, max_episode_steps: int | None = 100,
                 device: int | None = None, seed: int = 0, device_obs: bool = False, obs_dtype=None,
                 zero_copy: bool = False, **kwargs: Any):
        self.venv = PGTGVecEnv(num_envs, map_path, device=device, autoreset=True,
                               max_episode_steps=max_episode_steps, **kwargs)
        self.spec = self.venv.spec
        self.num_envs = num_envs
        self.obs_dim = flat_dim(self.spec)
        self._seed = seed
        self._actions = None
        self.device_obs = bool(device_obs)
        self.zero_copy = bool(zero_copy)
        self.obs_dtype = obs_dtype
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

    def _kernel_flat(self) -> bool:
        """The rows come from the HIP flattener (the host path's float32, the device path's float32 /
        int8); other device dtypes from flatten_obs."""
        import torch
        return not self.device_obs or self._dtype() in (torch.float32, torch.int8)

    def _bind_flat(self, final: bool):
        """Device rows for the next launch: fresh tensors on the device path (a step's tensors stay the
        caller's), one persistent pair on the host path (copied to the host before step_wait returns)."""
        import torch
        if not self.device_obs:
            if not hasattr(self, "_flat_d"):
                shape = (self.num_envs, self.obs_dim)
                self._flat_d = torch.empty(shape, dtype=torch.float32, device=self.venv.device)
                self._final_d = torch.empty(shape, dtype=torch.float32, device=self.venv.device)
                self.venv.set_flat_outputs(self._flat_d, self._final_d)
            return self._flat_d, self._final_d
        shape, dt = (self.num_envs, self.obs_dim), self._dtype()
        flat = torch.empty(shape, dtype=dt, device=self.venv.device)
        fin = torch.empty(shape, dtype=dt, device=self.venv.device) if final else None
        if getattr(self, "_flat_checked", None) == (dt, final):
            self.venv._bind_flat_ptrs(flat, fin, 0 if dt == torch.float32 else 1)
        else:  # (the first binding of this dtype and shape is checked)
            self.venv.set_flat_outputs(flat, fin)
            self._flat_checked = (dt, final)
        return flat, fin

    def reset(self):
        if self._kernel_flat():
            if self.device_obs:  # (the reset's observation pass must not write into the last step's scalars)
                self.venv.set_flat_scalars(None, None, None)
            flat, _ = self._bind_flat(final=False)
            self.venv.reset(seed=self._seed)
        else:
            obs, _ = self.venv.reset(seed=self._seed)
            flat = flatten_obs(self.spec, obs, dtype=self._dtype())
        return flat if self.device_obs else flat.cpu().numpy()

    def _dtype(self):
        import torch
        if self.obs_dtype is None:
            return torch.float32
        return getattr(torch, self.obs_dtype) if isinstance(self.obs_dtype, str) else self.obs_dtype

    def step_async(self, actions) -> None:
        import torch
        if isinstance(actions, torch.Tensor) and actions.device.type == "cuda":
            # device actions: no host round trip and no range check (that would be a device sync per
            # step); an action outside Discrete(9) is recorded by the kernel per env (error_count())
            a = actions.reshape(self.num_envs)
            if a.dtype != torch.uint8:  # every value outside Discrete(9) becomes the invalid code 255
                a = torch.where((a < 0) | (a > 8), torch.full_like(a, 255), a).to(torch.uint8)
            self._actions = a
            return
        a = np.asarray(actions.cpu() if isinstance(actions, torch.Tensor) else actions).reshape(self.num_envs)
        if a.size and (a.min() < 0 or a.max() > 8):  # an out-of-space action raises (environment.py:1118)
            raise KeyError(int(a[(a < 0) | (a > 8)][0]))
        self._actions = torch.as_tensor(a.astype(np.uint8))

    def step_wait(self):
        import torch
        kflat = self._kernel_flat()
        if kflat:  # the rows are written by k_flatten in the step: no torch work on the observations
            flat_d, final_d = self._bind_flat(final=True)
            if self.device_obs:  # ... nor on the rewards and done flags (written by the same pass)
                n, dev = self.num_envs, self.venv.device
                sc = (torch.empty(n, dtype=torch.float32, device=dev), torch.empty(n, dtype=torch.bool, device=dev),
                      torch.empty(n, dtype=torch.bool, device=dev))
                self.venv._bind_flat_scalar_ptrs(*sc)
            self.venv.step_launch(self._actions)
            v = self.venv
            reward, term, trunc, infos = v.reward, v.terminated, v.truncated, {}
            if v.cost is not None:
                infos["cost"] = v.cost
        else:
            obs, reward, term, trunc, infos = self.venv.step(self._actions)
        if self.device_obs and kflat:
            cost = infos.get("cost")
            if cost is not None:  # (the venv's output buffer, rewritten by the next step)
                cost = cost.clone()
            rew32, dones, tonly = sc
            return flat_d, rew32, dones, DeviceVecInfos(dones, tonly, final_d, cost)
        if self.device_obs:
            dones = term | trunc
            if kflat:
                flat, final = flat_d, final_d
            else:
                dt = self._dtype()
                flat = flatten_obs(self.spec, obs, dtype=dt)
                final = flatten_obs(self.spec, infos["final_observation"], dtype=dt)  # every row: no sync
            cost = infos.get("cost")
            if cost is not None:  # (the venv's output buffer, rewritten by the next step)
                cost = cost.clone()
            return (flat, reward.to(torch.float32), dones, DeviceVecInfos(dones, trunc & ~term, final, cost))
        # host arrays (SB3's VecEnv contract): one copy per step into page-locked buffers, and the
        # terminal observations of the finished envs only.  The buffers are fresh for every step (torch's
        # caching host allocator: a block returns to the cache only when the arrays over it are dropped),
        # so a caller may keep a step's arrays as long as it likes, as with SubprocVecEnv; zero_copy=True
        # reuses two buffer sets in turn instead (a step's arrays are then valid until the step after next)
        h = self._host_buffers()
        h["obs"].copy_(flat_d, non_blocking=True)
        h["rew"].copy_(reward.to(torch.float32), non_blocking=True)
        h["term"].copy_(term, non_blocking=True)
        h["trunc"].copy_(trunc, non_blocking=True)
        cost = None
        if "cost" in infos:
            h["cost"].copy_(infos["cost"], non_blocking=True)
        torch.cuda.current_stream(self.venv.device).synchronize()
        term_h, trunc_h = h["term"].numpy().astype(bool), h["trunc"].numpy().astype(bool)
        dones = term_h | trunc_h
        final, rows = None, None
        idx = np.nonzero(dones)[0]
        if idx.size:  # (k_flatten wrote the finished envs' rows)
            final = final_d.index_select(0, torch.as_tensor(idx, device=final_d.device)).cpu().numpy()
            rows = np.full(self.num_envs, -1, np.int64)
            rows[idx] = np.arange(idx.size)
        if "cost" in infos:
            cost = h["cost"].numpy().copy()
        return h["obs"].numpy(), h["rew"].numpy(), dones, VecInfos(dones, trunc_h & ~term_h, final, cost, rows)

    def _new_host_buffers(self) -> dict:
        import torch

        def pinned(shape, dtype):
            return torch.empty(shape, dtype=dtype, pin_memory=True)
        return {"obs": pinned((self.num_envs, self.obs_dim), torch.float32),
                "rew": pinned((self.num_envs,), torch.float32),
                "term": pinned((self.num_envs,), torch.uint8),
                "trunc": pinned((self.num_envs,), torch.uint8),
                "cost": pinned((self.num_envs,), torch.float64)}

    def _host_buffers(self) -> dict:
        if not self.zero_copy:
            return self._new_host_buffers()
        if not hasattr(self, "_hbuf"):
            self._hbuf = [self._new_host_buffers() for _ in range(2)]
            self._flip = 0
        self._flip ^= 1
        return self._hbuf[self._flip]

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
