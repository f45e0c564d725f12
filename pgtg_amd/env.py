"""Single-environment facade with the reference's `PGTGEnv` surface (pgtg/environment.py:297-1281).

`PGTGEnv(map_path=None, **kwargs)` takes the reference constructor's keyword arguments (validated
the same way, pgtg_amd/config.py) and runs ONE episode on the GPU through the same HIP kernels as
`PGTGVecEnv` (a batch of one, no auto-reset).  Returns follow the reference:

  reset(seed=None, options=None) -> (obs, info)                           environment.py:581-656
  step(action)                   -> (obs, reward, terminated, truncated, info)   :1092-1281

with `obs = {"position": int64[2], "velocity": int64[2], "map": {feature: int64[win][win]},
["next_subgoal_direction": int]}` (numpy, copied out of the device buffers) and `info = get_info()`
(:1538-1578).  A step after termination raises RuntimeError("Already done, step has no further
effect") like the reference (:1109-1110).  Differences, by design:
  * `obs["velocity"]` is a copy; the reference returns an alias of its internal state (:1462);
  * `reward` is always a Python float (the reference returns int 0 when nothing was scored);
  * rendering (pgtg/graphic.py) is out of scope: `render_mode` is validated and kept like the
    reference's (environment.py:790), but `render()` draws nothing and returns None.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from enum import Enum
from typing import Any, NamedTuple

import numpy as np

from . import config as _cfg
from .vector import PGTGVecEnv


class Position(NamedTuple):  # environment.py:33-35
    x: int
    y: int


class DriverProfile(Enum):  # environment.py:38-45
    CONSERVATIVE = "conservative"
    NORMAL = "normal"
    AGGRESSIVE = "aggressive"
    ELDERLY = "elderly"
    RECKLESS = "reckless"


@dataclass
class Car:  # environment.py:112-120 (a snapshot; appending one to env.cars adds it on the device)
    id: int
    position: Position
    route: str
    driver_profile: DriverProfile = DriverProfile.NORMAL
    patience_counter: int = 0
    last_action_delay: int = 0
    stuck_counter: int = 0


class CarList(list):
    """`env.cars`: the device car list as Car snapshots; `append` adds a car to the episode."""

    def __init__(self, env: "PGTGEnv", cars):
        super().__init__(cars)
        self._env = env

    def append(self, car: Car) -> None:  # noqa: D401
        prof = car.driver_profile.value if isinstance(car.driver_profile, DriverProfile) else str(car.driver_profile)
        self._env._vec.add_car(0, int(car.position[0]), int(car.position[1]), _cfg.ROUTES.index(car.route),
                               _cfg.DRIVER_PROFILES.index(prof), int(car.id))
        self._env._vec.observe()
        super().append(car)


_SQ_NAMES = {"wall": 1 << 32, "car_spawner": 1 << 37, "start": 1 << 38, "subgoal": 1 << 39,
             "used subgoal": 1 << 40, "final goal": 1 << 41, "ice": 1 << 42, "broken road": 1 << 43,
             "sand": 1 << 44, "traffic_light": 1 << 45}


class EpisodeMapView:
    """Read-only `env.map` (pgtg/map.py:8-184) over the device map's square feature words."""

    def __init__(self, words: np.ndarray):
        self._w = words
        self.width, self.height = words.shape

    def inside_map(self, x: int, y: int) -> bool:
        return 0 <= x < self.width and 0 <= y < self.height

    def get_features_at(self, x: int, y: int) -> set[str]:
        if not self.inside_map(x, y):
            raise ValueError("coordinates are outside the map")
        w = int(self._w[x, y])
        out = {n for n, b in _SQ_NAMES.items() if w & b}
        out |= {_cfg.LANES[k] for k in range(32) if (w >> k) & 1}
        return out

    def feature_at(self, x: int, y: int, features) -> bool:
        names = [features] if isinstance(features, str) else list(features)
        return not self.get_features_at(x, y).isdisjoint(names)


_AGENT_DIR_NAMES = ["south_to_north", "south_to_north", "west_to_east", "west_to_east",
                    "north_to_south", "north_to_south", "east_to_west", "east_to_west"]
SQ_SUBGOAL = 1 << 39
SQ_FINAL_GOAL = 1 << 41


def _spaces(spec: _cfg.EnvSpec):
    """gymnasium spaces of the reference (environment.py:415-441) when gymnasium is importable."""
    try:
        from gymnasium import spaces
    except ImportError:
        return None, None
    win = spec.window
    obs = {
        "position": spaces.MultiDiscrete([9, 9], dtype=np.int32),
        "velocity": spaces.Box(low=-99, high=99, shape=(2,), dtype=np.int32),
        "map": spaces.Dict({k: spaces.MultiBinary((win, win)) for k, _ in spec.channels}),
    }
    if spec.next_subgoal:
        obs["next_subgoal_direction"] = spaces.Discrete(9, start=-1)
    return spaces.Discrete(9), spaces.Dict(obs)


def compass_direction(squares: np.ndarray, x: int, y: int, window: int) -> int:
    """_get_subgoal_compass_directions (environment.py:1037-1090): index of the active compass
    direction [N, NE, E, SE, S, SW, W, NW] towards the nearest (Manhattan, x-major scan, strict <)
    subgoal / final-goal square, or -1 when there is none or it lies within `window` on both axes."""
    goal = (squares & np.uint64(SQ_SUBGOAL | SQ_FINAL_GOAL)) != 0
    xs, ys = np.nonzero(goal)  # x-major order, like the reference's nested loops
    if xs.size == 0:
        return -1
    d = np.abs(xs - x) + np.abs(ys - y)
    k = int(np.argmin(d))  # first minimum == strict < scan
    dx, dy = int(xs[k]) - x, int(ys[k]) - y
    if abs(dx) <= window and abs(dy) <= window:
        return -1
    a = math.atan2(dy, dx)
    p8 = math.pi / 8
    if -p8 <= a < p8:
        return 2
    if p8 <= a < 3 * p8:
        return 3
    if 3 * p8 <= a < 5 * p8:
        return 4
    if 5 * p8 <= a < 7 * p8:
        return 5
    if a >= 7 * p8 or a < -7 * p8:
        return 6
    if -7 * p8 <= a < -5 * p8:
        return 7
    if -5 * p8 <= a < -3 * p8:
        return 0
    return 1


class PGTGEnv:
    metadata = {"render_modes": []}

    def __init__(self, map_path: str | None = None, *, device: int | None = None, **kwargs: Any):
        self.spec = _cfg.make_spec(map_path, **kwargs)  # validates render_mode (environment.py:790)
        self.render_mode = self.spec.render_mode
        self.map_path = map_path
        # room for cars appended by hand (env.cars.append(Car(...)), as the reference tests do)
        self._vec = PGTGVecEnv(1, spec=self.spec, device=device, autoreset=False, min_car_capacity=64)
        self.action_space, self.observation_space = _spaces(self.spec)
        self.features_to_include_in_observation = [k for k, _ in self.spec.channels]
        self.terminated = False
        self.truncated = False
        self._reset_done = False
        self._triggered = 0

    # -- gymnasium API --------------------------------------------------------------------------
    def reset(self, *, seed: int | None = None, options: dict[str, Any] | None = None):
        self._vec.reset(seed=seed)
        self.terminated = self.truncated = False
        self._reset_done = True
        return self.get_observation(), self.get_info()

    def step(self, action: int):
        if not self._reset_done:
            raise RuntimeError("reset() must be called before step()")
        if self.terminated or self.truncated:
            raise RuntimeError("Already done, step has no further effect")
        a = int(action)
        if not 0 <= a < 9:
            raise KeyError(action)  # ACTIONS_TO_ACCELERATION[action] (environment.py:1118)
        _, reward, term, trunc, infos = self._vec.step(np.array([a], dtype=np.uint8))
        self.terminated = bool(term[0].item())
        self.truncated = bool(trunc[0].item())
        self._triggered = int(infos["triggered_rules_mask"][0].item())
        info = self.get_info()
        r = float(reward[0].item())
        if self.spec.separate_reward_cost:
            cost = float(infos["cost"][0].item())
            info["cost"] = cost
            info["performance_reward"] = r
            info["safety_cost"] = cost
        return self.get_observation(), r, self.terminated, self.truncated, info

    def close(self):
        self._vec.close()

    def light_step(self, action: int):
        """environment.py:1283-1299: a step on a copy; this env is unchanged afterwards.  The copy is
        the device state blob (pgtg_dump_state / pgtg_load_state), so RNG streams are restored too."""
        blob = self._vec.dump_state()
        flags = (self.terminated, self.truncated, self._triggered)
        try:
            out = self.step(action)
        finally:
            self._vec.load_state(blob)
            self.terminated, self.truncated, self._triggered = flags
        return out

    def set_to_state(self, state: dict[str, Any]):
        """environment.py:1301-1342: position, velocity, flat tire and the car list (patience and delay
        reset, unknown driver profiles -> normal, next car id = last id + 1); returns (obs, info)."""
        cars = []
        for cd in state.get("cars") or []:
            prof = cd.get("driver_profile", "normal")
            if prof not in _cfg.DRIVER_PROFILES:
                prof = "normal"
            cars.append((int(cd["id"]), int(cd["x"]), int(cd["y"]), _cfg.ROUTES.index(cd["route"]),
                         _cfg.DRIVER_PROFILES.index(prof)))
        self._vec.set_to_state(0, int(state["x"]), int(state["y"]), int(state["x_velocity"]),
                               int(state["y_velocity"]), bool(state["flat_tire"]), cars)
        self._vec.observe()
        return self.get_observation(), self.get_info()

    def save_map(self, path: str) -> None:
        """pgtg/map.py:173-184: the episode's map plan as JSON (loadable with map_path=)."""
        _cfg.save_map_plan(self._vec.map_plan(0), path)

    def render(self):
        """Frames (pgtg/graphic.py) are out of scope for this build: nothing is drawn."""
        return None

    # -- state ----------------------------------------------------------------------------------
    def get_observation(self) -> dict[str, Any]:
        v = self._vec
        obs: dict[str, Any] = {
            "position": v.position[0].cpu().numpy().astype(np.int64),
            "velocity": v.velocity[0].cpu().numpy().astype(np.int64),
            "map": {k: v.obs_map[0, i].cpu().numpy().astype(np.int64) for i, k in enumerate(v.keys)},
        }
        if v.nsd is not None:
            obs["next_subgoal_direction"] = int(v.nsd[0].item())
        return obs

    @property
    def position(self) -> np.ndarray:
        st = self._vec.env_state(0)
        return np.array([st["x"], st["y"]])

    @position.setter
    def position(self, xy) -> None:
        st = self._vec.env_state(0)
        self._vec.set_agent(0, int(xy[0]), int(xy[1]), st["vx"], st["vy"])
        self._vec.observe()

    @property
    def velocity(self) -> np.ndarray:
        st = self._vec.env_state(0)
        return np.array([st["vx"], st["vy"]])

    @velocity.setter
    def velocity(self, v) -> None:
        st = self._vec.env_state(0)
        self._vec.set_agent(0, st["x"], st["y"], int(v[0]), int(v[1]))
        self._vec.observe()

    @property
    def flat_tire(self) -> bool:
        return bool(self._vec.env_state(0)["flat_tire"])

    @property
    def cars(self) -> CarList:
        return CarList(self, [Car(int(c[0]), Position(int(c[1]), int(c[2])), _cfg.ROUTES[int(c[3])],
                                  DriverProfile(_cfg.DRIVER_PROFILES[int(c[4])]), int(c[5]), int(c[6]))
                              for c in self._vec.cars(0)])

    def _info_cars(self) -> list[dict[str, Any]]:
        return [{"id": c.id, "x": c.position.x, "y": c.position.y, "route": c.route,
                 "driver_profile": c.driver_profile.value, "patience_counter": c.patience_counter}
                for c in self.cars]

    @property
    def map(self) -> EpisodeMapView:
        return EpisodeMapView(self._vec.squares(0))

    @property
    def _next_car_id(self) -> int:
        return int(self._vec.env_state(0)["next_car_id"])

    def map_plan(self) -> dict:
        return self._vec.map_plan(0)

    def squares(self) -> np.ndarray:
        return self._vec.squares(0)

    def applicable_actions(self) -> list[int]:
        return [] if (self.terminated or self.truncated) else list(range(9))

    # -- traffic rules (environment.py:517-579) -------------------------------------------------
    def add_traffic_rule(self, rule_dict: dict[str, Any]) -> None:
        self._vec.add_traffic_rule(rule_dict)

    def remove_traffic_rule(self, rule_name: str) -> bool:
        return self._vec.remove_traffic_rule(rule_name)

    def get_agent_direction_string(self) -> str:
        st = self._vec.env_state(0)
        d = compass_direction(self._vec.squares(0), st["x"], st["y"], self.spec.sliding_size)
        if d >= 0:
            return _AGENT_DIR_NAMES[d]
        return "stationary" if math.hypot(st["vx"], st["vy"]) < 0.1 else "near_goal"

    # -- info (environment.py:1538-1578) --------------------------------------------------------
    def get_driver_profile_stats(self, cars: list[dict] | None = None) -> dict:
        cars = self._info_cars() if cars is None else cars
        counts = {p: 0 for p in _cfg.DRIVER_PROFILES}
        for c in cars:
            counts[c["driver_profile"]] += 1
        total = len(cars)
        pct = {k: (v / total) * 100 for k, v in counts.items()} if total else {k: 0 for k in counts}
        tot_cfg = sum(self.spec.profile_pct)
        return {"counts": counts, "percentages": pct, "total_cars": total,
                "configured_percentages": {p: v * 100 for p, v in zip(_cfg.DRIVER_PROFILES, self.spec.profile_pct)}
                if tot_cfg >= 0 else {}}

    def get_info(self) -> dict[str, Any]:
        st = self._vec.env_state(0)
        plan = self._vec.map_plan(0)
        tx = max(0, min(int(st["x"] // 9), plan["w"] - 1))
        ty = max(0, min(int(st["y"] // 9), plan["h"] - 1))
        ex = plan["exits"][ty * plan["w"] + tx]
        cars = self._info_cars() if st["n_cars"] else []
        names = self._vec.rule_names()
        return {
            "x": st["x"], "y": st["y"], "x_velocity": st["vx"], "y_velocity": st["vy"],
            "flat_tire": bool(st["flat_tire"]),
            "current_tile_type": "".join(str((ex >> d) & 1) for d in range(4)),
            "cars": cars,
            "driver_profile_stats": self.get_driver_profile_stats(cars),
            "traffic_rules": {
                "active_rules": list(names),
                "triggered_rules": [n for r, n in enumerate(names) if (self._triggered >> r) & 1],
                "braking_applied": self._triggered != 0,
                "agent_direction": self.get_agent_direction_string(),
            },
        }
