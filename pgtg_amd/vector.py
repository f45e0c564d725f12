"""Batched, device-resident PGTG environments (the MI355X hot path).

`PGTGVecEnv(num_envs, map_path=None, **PGTGEnv kwargs)` advances `num_envs` independent reference
episodes in lockstep on one GPU through the C ABI (include/pgtg.h) of `libpgtg_hip.so`.  Semantics
per env are the reference's `PGTGEnv.reset/step` (pgtg/environment.py:581-656, 1092-1281); the
batch follows the gymnasium/SB3 vector-env conventions: env i of a `reset(seed=s)` is seeded with
`s + i`, and an env that terminates (or is truncated by `max_episode_steps`, the TimeLimit wrapper
of pgtg/train.py:39) is reset unseeded in the same step, its terminal observation being returned
in `infos["final_observation"]`.

All returned tensors live on the GPU and are views of handle-owned buffers, valid until the next
call (clone them to keep them).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Any

from . import _abi
from .config import EnvSpec, make_spec

_EXC = {
    _abi.PGTG_E_INVALID: ValueError,
    _abi.PGTG_E_DONE: RuntimeError,
    _abi.PGTG_E_DEVICE: RuntimeError,
    _abi.PGTG_E_UNSUPPORTED: ValueError,
    _abi.PGTG_E_MAP: ValueError,
}


def _check(rc: int, handle=None) -> None:
    if rc != _abi.PGTG_OK:
        msg = _abi.lib().pgtg_last_error(handle)
        raise _EXC.get(rc, RuntimeError)((msg or b"").decode() or f"pgtg error {rc}")


class PGTGVecEnv:
    def __init__(self, num_envs: int, map_path: str | None = None, *, device: int | None = None,
                 autoreset: bool = True, max_episode_steps: int | None = None, spec: EnvSpec | None = None,
                 min_car_capacity: int = 0, tune: dict | None = None, **kwargs: Any):
        import torch

        self.spec = spec if spec is not None else make_spec(map_path, **kwargs)
        self.num_envs = int(num_envs)
        self.autoreset = autoreset
        self.max_episode_steps = max_episode_steps
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device)
        self._lib = _abi.lib()
        # tune: launch-shape overrides for tests/A-B runs (include/pgtg.h PgtgConfig.tune_*)
        self._cfg = _abi.config_struct(self.spec, autoreset, max_episode_steps, min_car_capacity, tune)
        h = C.c_void_p()
        _check(self._lib.pgtg_create(C.byref(self._cfg), self.num_envs, int(device), C.byref(h)), None)
        self._h = h
        self.window = self._lib.pgtg_window(h)
        self.keys = [k for k, _ in self.spec.channels]
        N, Cn, W = self.num_envs, len(self.keys), self.window
        dev = self.device
        t = torch
        self.obs_map = t.zeros((N, Cn, W, W), dtype=t.uint8, device=dev)
        self.position = t.zeros((N, 2), dtype=t.int32, device=dev)
        self.velocity = t.zeros((N, 2), dtype=t.int32, device=dev)
        self.reward = t.zeros((N,), dtype=t.float64, device=dev)
        self.terminated = t.zeros((N,), dtype=t.bool, device=dev)
        self.truncated = t.zeros((N,), dtype=t.bool, device=dev)
        self.braking = t.zeros((N,), dtype=t.uint8, device=dev)  # triggered-rule mask
        self.cost = t.zeros((N,), dtype=t.float64, device=dev) if self.spec.separate_reward_cost else None
        self.nsd = t.full((N,), -1, dtype=t.int32, device=dev) if self.spec.next_subgoal else None
        if autoreset:
            self.final_map = t.zeros_like(self.obs_map)
            self.final_position = t.zeros_like(self.position)
            self.final_velocity = t.zeros_like(self.velocity)
            self.final_nsd = t.full((N,), -1, dtype=t.int32, device=dev) if self.spec.next_subgoal else None
        else:
            self.final_map = self.final_position = self.final_velocity = self.final_nsd = None
        self.actions = t.zeros((N,), dtype=t.uint8, device=dev)
        o = _abi.PgtgOutputs()
        ptr = lambda x: None if x is None else x.data_ptr()  # noqa: E731
        o.obs, o.position, o.velocity = ptr(self.obs_map), ptr(self.position), ptr(self.velocity)
        o.next_subgoal, o.reward, o.cost = ptr(self.nsd), ptr(self.reward), ptr(self.cost)
        o.terminated, o.truncated, o.braking = ptr(self.terminated), ptr(self.truncated), ptr(self.braking)
        o.final_obs, o.final_position = ptr(self.final_map), ptr(self.final_position)
        o.final_velocity, o.final_next_subgoal = ptr(self.final_velocity), ptr(self.final_nsd)
        self._outs = o
        _check(self._lib.pgtg_set_outputs(h, C.byref(o)), h)
        self.has_cars = self.spec.traffic_density > 0 or min_car_capacity > 0  # the handle keeps car lists
        self._seeded = False

    # -- plumbing ------------------------------------------------------------------------------
    def _bind_stream(self):
        import torch
        s = torch.cuda.current_stream(self.device).cuda_stream
        if s != getattr(self, "_stream", None):  # (a ctypes call only when the stream changed)
            _check(self._lib.pgtg_set_stream(self._h, C.c_void_p(s)), self._h)
            self._stream = s

    def close(self):
        if getattr(self, "_h", None):
            self._lib.pgtg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def observation(self) -> dict:
        o = {"position": self.position, "velocity": self.velocity,
             "map": {k: self.obs_map[:, i] for i, k in enumerate(self.keys)}}
        if self.nsd is not None:
            o["next_subgoal_direction"] = self.nsd
        return o

    def final_observation(self) -> dict:
        o = {"position": self.final_position, "velocity": self.final_velocity,
             "map": {k: self.final_map[:, i] for i, k in enumerate(self.keys)}}
        if self.final_nsd is not None:
            o["next_subgoal_direction"] = self.final_nsd
        return o

    # -- API -----------------------------------------------------------------------------------
    def reset(self, *, seed: int | list[int] | None = None, options: dict | None = None,
              mask=None) -> tuple[dict, dict]:
        """Seeded reset: env i gets seed+i (or seed[i]); unseeded: next spawn block per env.
        `mask` (bool/uint8 [N] tensor) restricts the reset to some envs."""
        self._bind_stream()
        mptr = None
        if mask is not None:
            import torch
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
            self._mask = m
            mptr = C.c_void_p(m.data_ptr())
        if seed is None and not self._seeded:
            seed = int.from_bytes(os.urandom(7), "little")  # gymnasium: fresh OS entropy
        if seed is None:
            _check(self._lib.pgtg_reset_unseeded(self._h, mptr), self._h)
        elif isinstance(seed, int):
            if seed < 0:
                raise ValueError("seed must be a non-negative int")
            _check(self._lib.pgtg_reset(self._h, None, C.c_uint64(seed), mptr), self._h)
        else:
            seeds_l = [int(s) for s in seed]
            if len(seeds_l) != self.num_envs:
                raise ValueError(f"reset(seed=list) needs {self.num_envs} seeds, got {len(seeds_l)}")
            if any(s < 0 for s in seeds_l):
                raise ValueError("seed must be a non-negative int")
            seeds = (C.c_uint64 * self.num_envs)(*seeds_l)
            _check(self._lib.pgtg_reset(self._h, seeds, 0, mptr), self._h)
        self._seeded = True
        return self.observation(), {}

    def step(self, actions) -> tuple[dict, Any, Any, Any, dict]:
        self.step_launch(actions)
        infos: dict[str, Any] = {"braking_applied": self.braking != 0, "triggered_rules_mask": self.braking}
        if self.autoreset:
            done = self.terminated | self.truncated
            infos["final_observation"] = self.final_observation()
            infos["_final_observation"] = done
        if self.cost is not None:
            infos["cost"] = self.cost
        return self.observation(), self.reward, self.terminated, self.truncated, infos

    def step_launch(self, actions) -> None:
        """step() without building the returned dicts: the outputs are in the handle's tensors
        (obs_map, reward, terminated, truncated, final_map, ..., and any bound flat rows)."""
        import torch
        self._bind_stream()
        if not isinstance(actions, torch.Tensor):
            import numpy as np
            host = np.asarray(actions)
            if host.shape != (self.num_envs,):
                raise ValueError(f"expected {self.num_envs} actions, got shape {host.shape}")
            if host.size and (host.min() < 0 or host.max() > 8):  # Discrete(9): environment.py:1118
                raise KeyError(int(host[(host < 0) | (host > 8)][0]))
            actions = torch.as_tensor(host.astype(np.uint8))
        elif actions.numel() != self.num_envs:
            raise ValueError(f"expected {self.num_envs} actions, got {actions.numel()}")
        elif actions.dtype != torch.uint8 or actions.device.type != "cuda":
            # other dtypes / host tensors: range-checked here (a uint8 device tensor is not: the check
            # would be a device sync per step; the kernel records PGTG_E_INVALID per env instead, and
            # non-autoreset handles raise it below; autoreset callers read error_count())
            if bool(((actions < 0) | (actions > 8)).any()):
                raise KeyError("action outside Discrete(9)")
        a = actions
        if a.device != self.device or a.dtype != torch.uint8:
            a = a.to(device=self.device, dtype=torch.uint8)
        a = a.contiguous()
        self._act_ref = a
        _check(self._lib.pgtg_step(self._h, C.c_void_p(a.data_ptr())), self._h)
        if not self.autoreset:
            self._raise_errors()

    def step_random(self, seed: int, t: int, env_offset: int = 0):
        """One tick with device-generated uniform random actions (synthetic rollouts, bench)."""
        self._bind_stream()
        _check(self._lib.pgtg_random_actions(self._h, C.c_void_p(self.actions.data_ptr()), C.c_uint64(seed),
                                             C.c_uint64(t), C.c_uint64(env_offset)), self._h)
        _check(self._lib.pgtg_step(self._h, C.c_void_p(self.actions.data_ptr())), self._h)

    def random_actions(self, steps: int, seed: int, t0: int = 0, env_offset: int = 0):
        """[steps, N] uint8 device tensor of synthetic uniform actions (the same hash as step_random),
        generated ahead so that a timed rollout starts with its inputs resident in HBM.  `env_offset`
        is the global index of env 0 (sharded runs draw the actions of the whole batch's envs)."""
        import torch
        self._bind_stream()
        a = torch.empty((steps, self.num_envs), dtype=torch.uint8, device=self.device)
        for k in range(steps):
            _check(self._lib.pgtg_random_actions(self._h, C.c_void_p(a[k].data_ptr()), C.c_uint64(seed),
                                                 C.c_uint64(t0 + k), C.c_uint64(env_offset)), self._h)
        return a

    def step_actions(self, actions_row):
        """One tick from a resident [N] uint8 device tensor, no host conversion or returned views."""
        self._bind_stream()
        _check(self._lib.pgtg_step(self._h, C.c_void_p(actions_row.data_ptr())), self._h)

    def step_many(self, actions):
        """len(actions) ticks from a resident [T, N] uint8 device tensor in one host call
        (include/pgtg.h pgtg_step_many); the outputs hold the last tick's."""
        import torch
        if actions.dim() != 2 or actions.shape[1] != self.num_envs or actions.dtype != torch.uint8:
            raise ValueError(f"expected a [T, {self.num_envs}] uint8 tensor, got {tuple(actions.shape)} {actions.dtype}")
        if actions.device != self.device or actions.stride(1) != 1:
            raise ValueError("actions must be a row-contiguous tensor on the env's device")
        self._bind_stream()
        _check(self._lib.pgtg_step_many(self._h, C.c_void_p(actions.data_ptr()), actions.stride(0),
                                        actions.shape[0]), self._h)

    def set_flat_outputs(self, flat=None, final_flat=None):
        """Have every launch also write the FlattenObservation rows (pgtg/train.py:40) of the
        observation into `flat` and, in steps, the finished envs' terminal rows into `final_flat`:
        [N, flat_dim] float32 or int8 device tensors (include/pgtg.h pgtg_set_flat_outputs; the HIP
        kernel k_flatten, no torch work).  Rebinding per step is cheap (the pointers are kept by the
        handle); None, None turns it off."""
        import torch

        from .flat import check_flattenable, flat_dim, flat_order
        bufs = [t for t in (flat, final_flat) if t is not None]
        if not bufs:
            _check(self._lib.pgtg_set_flat_outputs(self._h, None, 0, 0, None, None), self._h)
            self._flat_refs = ()
            return
        check_flattenable(self.spec)
        D = flat_dim(self.spec)
        dt = bufs[0].dtype
        for t in bufs:
            if t.dtype not in (torch.float32, torch.int8) or t.dtype != dt:
                raise ValueError("flat rows: float32 or int8 tensors, both of one dtype")
            if tuple(t.shape) != (self.num_envs, D) or not t.is_contiguous() or t.device != self.device:
                raise ValueError(f"flat rows: contiguous [{self.num_envs}, {D}] tensors on {self.device}")
        if final_flat is not None and not self.autoreset:
            raise ValueError("terminal flat rows need autoreset=True")
        order = flat_order(self.spec)
        self._flat_order = (C.c_int32 * len(order))(*order)
        self._bind_flat_ptrs(flat, final_flat, 0 if dt == torch.float32 else 1)

    def set_flat_scalars(self, reward_f32=None, dones=None, truncated_only=None) -> None:
        """With flat rows bound, every observation pass also writes the reward as float32, done =
        terminated | truncated and truncated-and-not-terminated into these [N] device tensors (float32,
        bool, bool; include/pgtg.h pgtg_set_flat_scalars).  None, None, None unbinds."""
        import torch
        ts = (reward_f32, dones, truncated_only)
        if all(t is None for t in ts):
            _check(self._lib.pgtg_set_flat_scalars(self._h, None, None, None), self._h)
            self._flat_scalar_refs = ()
            return
        if any(t is None for t in ts):
            raise ValueError("flat scalars: all three tensors or none")
        for t, dt in zip(ts, (torch.float32, torch.bool, torch.bool)):
            if t.dtype != dt or tuple(t.shape) != (self.num_envs,) or not t.is_contiguous() or t.device != self.device:
                raise ValueError(f"flat scalars: contiguous [{self.num_envs}] {dt} tensors on {self.device}")
        self._bind_flat_scalar_ptrs(*ts)

    def _bind_flat_scalar_ptrs(self, reward_f32, dones, truncated_only) -> None:
        _check(self._lib.pgtg_set_flat_scalars(self._h, C.c_void_p(reward_f32.data_ptr()), C.c_void_p(dones.data_ptr()),
                                               C.c_void_p(truncated_only.data_ptr())), self._h)
        self._flat_scalar_refs = (reward_f32, dones, truncated_only)

    def _bind_flat_ptrs(self, flat, final_flat, dtype_code: int) -> None:
        """Rebind flat rows already checked by set_flat_outputs (same shape and dtype): the per-step
        path of PGTGSB3VecEnv, which hands out fresh tensors every step."""
        ptr = lambda x: None if x is None else C.c_void_p(x.data_ptr())  # noqa: E731
        _check(self._lib.pgtg_set_flat_outputs(self._h, self._flat_order, len(self._flat_order), dtype_code,
                                               ptr(flat), ptr(final_flat)), self._h)
        self._flat_refs = (flat, final_flat)  # (the handle writes into them: keep them alive)

    def observe(self):
        """Re-emit every env's observation (after set_agent / add_car)."""
        self._bind_stream()
        _check(self._lib.pgtg_observe(self._h), self._h)
        return self.observation()

    def error_count(self) -> tuple[int, int]:
        """(envs whose last step failed, first error code); e.g. PGTG_E_INVALID for an action > 8
        passed in a uint8 device tensor, which step() does not range-check."""
        n = C.c_uint64()
        code = C.c_int32()
        _check(self._lib.pgtg_error_count(self._h, C.byref(n), C.byref(code)), self._h)
        return n.value, code.value

    def _raise_errors(self):
        n = C.c_uint64()
        code = C.c_int32()
        _check(self._lib.pgtg_error_count(self._h, C.byref(n), C.byref(code)), self._h)
        if n.value:
            if code.value == _abi.PGTG_E_DONE:
                raise RuntimeError("Already done, step has no further effect")
            raise _EXC.get(code.value, RuntimeError)(f"{n.value} env(s) failed with code {code.value}")

    # -- introspection (host-synchronising) ------------------------------------------------------
    def env_state(self, i: int) -> dict:
        st = _abi.PgtgEnvState()
        _check(self._lib.pgtg_get_env_state(self._h, i, C.byref(st)), self._h)
        d = {f: getattr(st, f) for f, _ in st._fields_}
        d["used_subgoals"] = sum(int(w) << (64 * k) for k, w in enumerate(st.used_subgoals))  # bit t: tile t
        return d

    def cars(self, i: int):
        import numpy as np
        n = C.c_int32()
        _check(self._lib.pgtg_get_cars(self._h, i, None, 0, C.byref(n)), self._h)
        arr = (_abi.PgtgCar * max(n.value, 1))()
        _check(self._lib.pgtg_get_cars(self._h, i, arr, n.value, C.byref(n)), self._h)
        return np.array([[c.id, c.x, c.y, c.route, c.profile, c.patience, c.delay] for c in arr[:n.value]],
                        dtype=np.int32).reshape(n.value, 7)

    def map_plan(self, i: int) -> dict:
        w, h = C.c_int32(), C.c_int32()
        ex = (C.c_uint8 * _abi.MAX_TILES)()
        ot = (C.c_int8 * _abi.MAX_TILES)()
        om = (C.c_int8 * _abi.MAX_TILES)()
        s3 = (C.c_int32 * 3)()
        g3 = (C.c_int32 * 3)()
        _check(self._lib.pgtg_get_map_plan(self._h, i, C.byref(w), C.byref(h), ex, ot, om, s3, g3), self._h)
        n = w.value * h.value
        return {"w": w.value, "h": h.value, "exits": list(ex[:n]), "otype": list(ot[:n]), "omask": list(om[:n]),
                "start": tuple(s3), "goal": tuple(g3)}

    def squares(self, i: int):
        """Feature words of env i's map squares, numpy uint64 [W*9][H*9] (include/pgtg.h PGTG_SQ_*)."""
        import numpy as np
        w, h = C.c_int32(), C.c_int32()
        _check(self._lib.pgtg_get_squares(self._h, i, None, 0, C.byref(w), C.byref(h)), self._h)
        out = np.zeros(w.value * h.value, np.uint64)
        _check(self._lib.pgtg_get_squares(self._h, i, C.c_void_p(out.ctypes.data), out.size, C.byref(w),
                                          C.byref(h)), self._h)
        return out.reshape(w.value, h.value)

    # -- traffic rules (TrafficRuleEngine via PGTGEnv.add_traffic_rule / remove_traffic_rule) ---------
    def _push_rules(self):
        arr = (_abi.PgtgRule * _abi.MAX_RULES)()
        n = _abi.fill_rules(arr, self.spec.rules)
        _check(self._lib.pgtg_set_rules(self._h, arr, n), self._h)

    def add_traffic_rule(self, rule_dict: dict):
        from .config import add_rule
        add_rule(self.spec, rule_dict)
        self._push_rules()

    def remove_traffic_rule(self, rule_name: str) -> bool:
        from .config import remove_rule
        removed = remove_rule(self.spec, rule_name)
        if removed:
            self._push_rules()
        return removed

    def rule_names(self) -> list[str]:
        return [r.name for r in self.spec.rules]

    # -- whole-batch state (bit-exact replay) and set_to_state --------------------------------------
    def dump_state(self):
        """Every env's device state as one uint8 numpy blob (include/pgtg.h pgtg_dump_state)."""
        import numpy as np
        n = C.c_uint64()
        _check(self._lib.pgtg_state_size(self._h, C.byref(n)), self._h)
        buf = np.empty(n.value, dtype=np.uint8)
        _check(self._lib.pgtg_dump_state(self._h, C.c_void_p(buf.ctypes.data), n.value), self._h)
        return buf

    def load_state(self, blob, observe: bool = True):
        """Restore a dump_state() blob of a handle with the same config and batch size; re-emits the
        observations unless observe=False."""
        import numpy as np
        b = np.ascontiguousarray(blob, dtype=np.uint8)
        _check(self._lib.pgtg_load_state(self._h, C.c_void_p(b.ctypes.data), b.size), self._h)
        self._seeded = True
        if observe:
            self.observe()

    def set_to_state(self, i: int, x: int, y: int, vx: int, vy: int, flat_tire: bool, cars=()):
        """PGTGEnv.set_to_state for env i (environment.py:1301-1342); cars = [(id, x, y, route, profile)]."""
        cars = list(cars)
        arr = (_abi.PgtgCar * max(1, len(cars)))()
        for k, (cid, cx, cy, route, prof) in enumerate(cars):
            arr[k].id, arr[k].x, arr[k].y, arr[k].route, arr[k].profile = int(cid), int(cx), int(cy), int(route), int(prof)
        _check(self._lib.pgtg_set_to_state(self._h, i, int(x), int(y), int(vx), int(vy), int(bool(flat_tire)), arr,
                                           len(cars)), self._h)

    def set_agent(self, i: int, x: int, y: int, vx: int, vy: int):
        _check(self._lib.pgtg_set_agent(self._h, i, x, y, vx, vy), self._h)

    def add_car(self, i: int, x: int, y: int, route: int, profile: int, car_id: int = -1):
        """Append a car to env i (car_id < 0: the env's next id)."""
        _check(self._lib.pgtg_add_car(self._h, i, x, y, route, profile, car_id), self._h)

    def mean_cars(self, sample: int = 64) -> float:
        """Average car count over (up to) `sample` envs (host-synchronising)."""
        idx = range(0, self.num_envs, max(1, self.num_envs // sample))
        return sum(self.env_state(i)["n_cars"] for i in idx) / len(idx)

    def launch_info(self) -> tuple[int, int]:
        """(envs per workgroup, LDS bytes per workgroup) of the step kernel."""
        e, b = C.c_int32(), C.c_int32()
        _check(self._lib.pgtg_launch_info(self._h, C.byref(e), C.byref(b)), self._h)
        return e.value, b.value

    def occupancy(self) -> int:
        """Workgroups of the step kernel resident per CU (HIP occupancy query)."""
        n = C.c_int32()
        _check(self._lib.pgtg_occupancy(self._h, C.byref(n)), self._h)
        return n.value

    def step_kernel(self) -> str:
        """Name of the kernel(s) a step launches (measurement labels)."""
        return self._lib.pgtg_step_kernel(self._h).decode()

    def car_digest(self):
        """Per-env digest of the car lists (int64 [N] device tensor; pgtg_amd/digest.py car_term)."""
        import torch
        out = torch.empty(self.num_envs, dtype=torch.int64, device=self.device)
        self._bind_stream()
        _check(self._lib.pgtg_car_digest(self._h, C.c_void_p(out.data_ptr())), self._h)
        return out

    def counters(self) -> tuple[int, int]:
        a, b = C.c_uint64(), C.c_uint64()
        _check(self._lib.pgtg_get_counters(self._h, C.byref(a), C.byref(b)), self._h)
        return a.value, b.value

    def queue_maps(self) -> int:
        """Map-queue ring entries generated since create (0 without the queue)."""
        m = C.c_uint64()
        _check(self._lib.pgtg_get_queue_maps(self._h, C.byref(m)), self._h)
        return m.value

    def queue_overflow(self) -> int:
        """Map-queue refill requests served from the one-round overflow lists since create."""
        m = C.c_uint64()
        if not hasattr(self._lib, "pgtg_get_queue_overflow"):  # (an older build, tools/ab_multi.sh)
            return -1
        _check(self._lib.pgtg_get_queue_overflow(self._h, C.byref(m)), self._h)
        return m.value

    def enable_timing(self, every: int = 1):
        """Bracket every `every`-th step launch with a HIP event pair (0: off)."""
        self._lib.pgtg_enable_timing(self._h, int(every))

    def timing_read(self, reset: bool = True) -> tuple[float, int]:
        """(summed step-kernel ms, timed launches) from HIP events on the handle's stream."""
        ms, n = C.c_double(), C.c_uint64()
        _check(self._lib.pgtg_timing_read(self._h, C.byref(ms), C.byref(n), int(reset)), self._h)
        return ms.value, n.value
