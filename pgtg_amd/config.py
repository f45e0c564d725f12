"""Host-side configuration: the reference's ~40 constructor kwargs frozen into a canonical
`EnvSpec` (validated exactly where the reference validates, raising the same exception types).

Mirrors `PGTGEnv.__init__` (/root/reference pgtg/environment.py:302-515), the start/goal checks of
`generate_map` (pgtg/map_generator.py:92-154), the JSON map loader (pgtg/parser.py:227-241) and
the default traffic rules (pgtg/environment.py:517-567).  Both the HIP product (via the C-ABI
struct in `pgtg_amd/_abi.py`) and the CPU oracle used by the tests are fed from an `EnvSpec`.
"""
from __future__ import annotations

import json
import math
import warnings
from dataclasses import dataclass, field
from typing import Any

TILE = 9
DIRECTIONS = ["north", "east", "south", "west"]  # pgtg/constants.py:31-36
OBSTACLE_NAMES = ["ice", "broken road", "sand", "traffic_light"]  # pgtg/constants.py:18
OBSTACLE_MASK_NAMES = [  # id order used by the tables (tools/gen_tables.py)
    "blob", "small_blob", "chess_field", "reverse_chess_field", "top_half", "bottom_half",
    "left_half", "right_half", "traffic_light_north", "traffic_light_east", "traffic_light_south",
    "traffic_light_west", "traffic_light_north_and_south", "traffic_light_east_and_west",
]
ROUTES = [
    "east_to_middle", "east_to_north", "east_to_south", "east_to_west", "middle_to_east",
    "middle_to_north", "middle_to_south", "middle_to_west", "north_to_east", "north_to_middle",
    "north_to_south", "north_to_west", "south_to_east", "south_to_middle", "south_to_north",
    "south_to_west", "west_to_east", "west_to_middle", "west_to_north", "west_to_south",
]
LANES = [
    "car_lane east_to_middle left", "car_lane east_to_north left", "car_lane east_to_north up",
    "car_lane east_to_south down", "car_lane east_to_south left", "car_lane east_to_west left",
    "car_lane middle_to_east right", "car_lane middle_to_north up", "car_lane middle_to_south down",
    "car_lane middle_to_west left", "car_lane north_to_east down", "car_lane north_to_east right",
    "car_lane north_to_middle down", "car_lane north_to_south down", "car_lane north_to_west down",
    "car_lane north_to_west left", "car_lane south_to_east right", "car_lane south_to_east up",
    "car_lane south_to_middle up", "car_lane south_to_north up", "car_lane south_to_west left",
    "car_lane south_to_west up", "car_lane west_to_east right", "car_lane west_to_middle right",
    "car_lane west_to_north right", "car_lane west_to_north up", "car_lane west_to_south down",
    "car_lane west_to_south right", "car_lane all up", "car_lane all down", "car_lane all left",
    "car_lane all right",
]
DRIVER_PROFILES = ["conservative", "normal", "aggressive", "elderly", "reckless"]
AGENT_DIRECTIONS = ["south_to_north", "west_to_east", "north_to_south", "east_to_west",
                    "stationary", "near_goal"]

# observation channel codes (include/pgtg.h PGTG_CH_*)
CH_ZERO, CH_WALL, CH_GOALS, CH_TRAFFIC, CH_TL_GREEN, CH_TL_YELLOW, CH_TL_RED = range(7)
CH_START, CH_SUBGOAL, CH_USED_SUBGOAL, CH_FINAL_GOAL, CH_ICE, CH_BROKEN, CH_SAND, CH_SPAWNER = range(7, 15)
CH_LANE0 = 32
_GENERIC = {
    "wall": CH_WALL, "start": CH_START, "subgoal": CH_SUBGOAL, "used subgoal": CH_USED_SUBGOAL,
    "final goal": CH_FINAL_GOAL, "ice": CH_ICE, "broken road": CH_BROKEN, "sand": CH_SAND,
    "car_spawner": CH_SPAWNER,
}
_GENERIC.update({name: CH_LANE0 + i for i, name in enumerate(LANES)})

DEFAULT_FEATURES = ["walls", "goals", "ice", "broken road", "sand", "traffic",
                    "traffic_light_green", "traffic_light_yellow", "traffic_light_red"]

# pgtg/environment.py:517-567
DEFAULT_RULES = [
    {
        "name": "four_way_intersection_brake", "tile_type": "1111", "velocity_range": [0.5, 10.0],
        "min_traffic": 1, "min_matching_traffic": 1,
        "maneuvers": [
            {"agent": "west_to_east", "traffic": ["north_to_south", "south_to_north"]},
            {"agent": "east_to_west", "traffic": ["north_to_south", "south_to_north"]},
            {"agent": "north_to_south", "traffic": ["west_to_east", "east_to_west"]},
            {"agent": "south_to_north", "traffic": ["west_to_east", "east_to_west"]},
        ],
    },
    {
        "name": "t_intersection_brake", "tile_type": "1110", "velocity_range": [0.5, 10.0],
        "min_traffic": 1, "min_matching_traffic": 1,
        "maneuvers": [
            {"agent": "south_to_north", "traffic": ["west_to_east", "east_to_west"]},
            {"agent": "west_to_east", "traffic": ["south_to_north"]},
        ],
    },
]
MAX_RULES = 8
MAX_CHANNELS = 128


def feature_channels(features: list[str]) -> list[tuple[str, int]]:
    """Ordered (key, channel code) list reproducing the keys of the reference's obs["map"] dict
    (pgtg/environment.py:1387-1445): walls/goals/traffic are special, "traffic_light" expands
    into the three phase keys, every other name is a one-hot of squares holding that feature
    (unknown names give all-zero channels; the generic pass runs last so it overwrites)."""
    keys: dict[str, int] = {}
    if "walls" in features:
        keys["walls"] = CH_WALL
    if "goals" in features:
        keys["goals"] = CH_GOALS
    if "traffic" in features:
        keys["traffic"] = CH_TRAFFIC
    if "traffic_light" in features:
        keys["traffic_light_green"] = CH_TL_GREEN
        keys["traffic_light_yellow"] = CH_TL_YELLOW
        keys["traffic_light_red"] = CH_TL_RED
    for f in features:
        if f in ("walls", "goals", "traffic", "traffic_light"):
            continue
        keys[f] = _GENERIC.get(f, CH_ZERO)
    order: list[str] = []
    for f in features:
        for k in (["traffic_light_green", "traffic_light_yellow", "traffic_light_red"]
                  if f == "traffic_light" else [f]):
            if k in keys and k not in order:
                order.append(k)
    return [(k, keys[k]) for k in order]


def _speed_sq_bounds(lo: float, hi: float, vmax: int = 1 << 15) -> tuple[int, int]:
    """Integer interval [smin, smax] of s = vx^2+vy^2 with lo <= sqrt(s) <= hi in fp64
    (np.linalg.norm of the int velocity, pgtg/environment.py:245-246).  sqrt is correctly rounded
    and monotone, so the admissible s form an interval; smax < smin encodes 'never'."""
    top = 2 * vmax * vmax

    def first_true(pred):  # smallest s in [0, top+1] with pred(s), pred monotone False->True
        a, b = -1, top + 1
        while a + 1 < b:
            m = (a + b) // 2
            if pred(m):
                b = m
            else:
                a = m
        return b

    smin = first_true(lambda s: lo <= math.sqrt(s))
    smax = first_true(lambda s: math.sqrt(s) > hi) - 1
    return smin, smax


@dataclass
class CompiledRule:
    name: str
    tile_exits: int  # exit mask, -1 never matches
    vel_lo: float
    vel_hi: float
    speed_sq_min: int
    speed_sq_max: int
    min_traffic: int
    min_matching_traffic: int
    weight: list[list[int]]  # [6 agent dirs][20 routes]


def compile_rule(rule: dict[str, Any]) -> CompiledRule:
    """TrafficRule.from_dict + evaluate_rule semantics (pgtg/environment.py:141-159, 226-273)."""
    tt = rule["tile_type"]
    if isinstance(tt, str) and len(tt) == 4 and set(tt) <= {"0", "1"}:
        mask = sum(1 << i for i, ch in enumerate(tt) if ch == "1")
    else:
        mask = -1
    lo, hi = float(rule["velocity_range"][0]), float(rule["velocity_range"][1])
    w = [[0] * len(ROUTES) for _ in AGENT_DIRECTIONS]
    for m in rule["maneuvers"]:
        if m["agent"] in AGENT_DIRECTIONS:
            d = AGENT_DIRECTIONS.index(m["agent"])
            for r, rname in enumerate(ROUTES):
                if rname in m["traffic"]:
                    w[d][r] += 1
    smin, smax = _speed_sq_bounds(lo, hi)
    return CompiledRule(rule["name"], mask, lo, hi, smin, smax, int(rule["min_traffic"]),
                        int(rule["min_matching_traffic"]), w)


def _parse_position(pos, name: str, width: int, height: int):
    """(mode, x, y, dir) from a start/goal kwarg; validation of pgtg/map_generator.py:92-126."""
    if isinstance(pos, str):
        if pos != "random":
            raise ValueError(f"{name} must be a tuple or 'random'.")
        return 2, 0, 0, -1
    pos = tuple(pos)
    if not (pos[0] == 0 or pos[0] == -1 or pos[0] == width - 1 or pos[1] == 0 or pos[1] == -1
            or pos[1] == height - 1):
        raise ValueError(f"{name} must specify a tile on the map border.")
    if len(pos) == 3:
        d = pos[2]
        ok = ((d != "north" or pos[1] == 0)
              and (d != "east" or (pos[0] == -1 or pos[0] == width - 1))
              and (d != "south" or (pos[1] == -1 or pos[1] == height - 1))
              and (d != "west" or pos[0] == 0))
        if not ok:
            raise ValueError(f"The direction in {name} is not a map border.")
        return 0, int(pos[0]), int(pos[1]), DIRECTIONS.index(d)
    return 1, int(pos[0]), int(pos[1]), -1


@dataclass
class MapPlanArrays:
    """A MapPlan (pgtg/map_generator.py:9-40) as flat row-major arrays."""
    width: int
    height: int
    exits: list[int]  # bit0 N, bit1 E, bit2 S, bit3 W
    obstacle_type: list[int]  # -1 none, index into OBSTACLE_NAMES
    obstacle_mask: list[int]  # -1 none, index into OBSTACLE_MASK_NAMES
    start: tuple[int, int, int]
    goal: tuple[int, int, int]

    @classmethod
    def from_dict(cls, data: dict[str, Any]) -> "MapPlanArrays":
        w, h = int(data["width"]), int(data["height"])
        tiles = data["map"]
        start, goal = data["start"], data["goal"]  # KeyError on the old format, like the reference
        ex, ot, om = [], [], []
        for y in range(h):
            for x in range(w):
                t = tiles[y][x]
                ex.append(sum(int(b) << i for i, b in enumerate(t["exits"])))
                otype = t.get("obstacle_type")
                if otype is not None:
                    if t.get("obstacle_mask") is None:
                        raise AssertionError(
                            f"The tile at ({x},{y}) has a obstacle type without a obstacle mask")
                    if otype not in OBSTACLE_NAMES:
                        raise AssertionError(f"Unknown obstacle type: {otype}")
                    ot.append(OBSTACLE_NAMES.index(otype))
                    om.append(OBSTACLE_MASK_NAMES.index(t["obstacle_mask"]))
                else:
                    ot.append(-1)
                    om.append(-1)
        return cls(w, h, ex, ot, om, (int(start[0]), int(start[1]), DIRECTIONS.index(start[2])),
                   (int(goal[0]), int(goal[1]), DIRECTIONS.index(goal[2])))

    def to_dict(self) -> dict[str, Any]:
        rows = []
        for y in range(self.height):
            row = []
            for x in range(self.width):
                i = y * self.width + x
                t: dict[str, Any] = {"exits": [(self.exits[i] >> b) & 1 for b in range(4)]}
                if self.obstacle_type[i] >= 0:
                    t["obstacle_type"] = OBSTACLE_NAMES[self.obstacle_type[i]]
                    t["obstacle_mask"] = OBSTACLE_MASK_NAMES[self.obstacle_mask[i]]
                row.append(t)
            rows.append(row)
        return {"width": self.width, "height": self.height, "map": rows,
                "start": [self.start[0], self.start[1], DIRECTIONS[self.start[2]]],
                "goal": [self.goal[0], self.goal[1], DIRECTIONS[self.goal[2]]]}


def save_map_plan(plan: dict, path: str) -> None:
    """EpisodeMap.save_map (pgtg/map.py:173-184): a device map plan (PGTGVecEnv.map_plan) as the
    reference's JSON (MapPlan.to_dict, pgtg/map_generator.py:31-40; '.json' appended when missing)."""
    n = plan["w"] * plan["h"]
    mp = MapPlanArrays(plan["w"], plan["h"], list(plan["exits"][:n]), list(plan["otype"][:n]),
                       list(plan["omask"][:n]), tuple(plan["start"]), tuple(plan["goal"]))
    if not path.endswith(".json"):
        path += ".json"
    with open(path, "w", encoding="utf-8") as f:
        json.dump(mp.to_dict(), f, ensure_ascii=False, indent=4)


def json_file_to_map_plan(path: str) -> MapPlanArrays:
    """pgtg/parser.py:227-241."""
    if not path.endswith(".json"):
        path = path + ".json"
    with open(path) as f:
        return MapPlanArrays.from_dict(json.load(f))


@dataclass
class EnvSpec:
    width: int = 4
    height: int = 4
    pct_connections: float = 0.5
    start_mode: int = 0
    start_xyd: tuple[int, int, int] = (0, -1, 3)
    goal_mode: int = 0
    goal_xyd: tuple[int, int, int] = (-1, 0, 1)
    min_distance: int = -1
    obstacle_probability: float = 0.0
    weights: tuple[float, float, float, float] = (1.0, 1.0, 1.0, 1.0)
    features: list[str] = field(default_factory=lambda: list(DEFAULT_FEATURES))
    channels: list[tuple[str, int]] = field(default_factory=list)
    sliding: bool = False
    sliding_size: int = 4
    next_subgoal: bool = False
    sum_subgoals_reward: float = 100
    final_goal_bonus: float = 0
    crash_penalty: float = 100
    tl_violation_penalty: float = 50
    standing_still_penalty: float = 0
    visited_penalty: float = 0
    ice_probability: float = 0.1
    street_damage_probability: float = 0.1
    sand_probability: float = 0.2
    traffic_density: float = 0.0
    phase_dur: tuple[int, int, int] = (10, 3, 10)
    ignore_traffic_collisions: bool = False
    max_allowed_deviation: int | None = 10
    profile_pct: tuple[float, ...] = (0.25, 0.35, 0.20, 0.15, 0.05)
    separate_reward_cost: bool = False
    rules: list[CompiledRule] = field(default_factory=list)
    fixed_map: MapPlanArrays | None = None
    map_path: str | None = None
    render_mode: str | None = None

    @property
    def window(self) -> int:
        return 1 + 2 * self.sliding_size if self.sliding else TILE

    @property
    def map_tiles(self) -> tuple[int, int]:
        if self.fixed_map is not None:
            return self.fixed_map.width, self.fixed_map.height
        return self.width, self.height


def make_spec(map_path: str | None = None, **kw: Any) -> EnvSpec:
    """`PGTGEnv(map_path, **kwargs)` -> EnvSpec; unknown kwargs raise TypeError like a Python call."""
    allowed = {
        "random_map_width", "random_map_height", "random_map_percentage_of_connections",
        "random_map_start_position", "random_map_goal_position",
        "random_map_minimum_distance_between_start_and_goal", "random_map_obstacle_probability",
        "random_map_ice_probability_weight", "random_map_broken_road_probability_weight",
        "random_map_sand_probability_weight", "random_map_traffic_light_probability_weight",
        "render_mode", "features_to_include_in_observation", "use_sliding_observation_window",
        "sliding_observation_window_size", "use_next_subgoal_direction", "sum_subgoals_reward",
        "final_goal_bonus", "crash_penalty", "traffic_light_violation_penalty",
        "standing_still_penalty", "already_visited_position_penalty", "ice_probability",
        "street_damage_probability", "sand_probability", "traffic_density",
        "traffic_light_phases_duration", "ignore_traffic_collisions", "max_allowed_deviation",
        "conservative_driver_percentage", "normal_driver_percentage",
        "aggressive_driver_percentage", "elderly_driver_percentage",
        "reckless_driver_percentage", "separate_reward_cost",
    }
    bad = set(kw) - allowed
    if bad:
        raise TypeError(f"PGTGEnv.__init__() got an unexpected keyword argument '{sorted(bad)[0]}'")
    g = kw.get
    s = EnvSpec()
    s.width = int(g("random_map_width", 4))
    s.height = int(g("random_map_height", 4))
    s.pct_connections = float(g("random_map_percentage_of_connections", 0.5))
    s.obstacle_probability = float(g("random_map_obstacle_probability", 0.0))
    s.weights = (g("random_map_ice_probability_weight", 1), g("random_map_broken_road_probability_weight", 1),
                 g("random_map_sand_probability_weight", 1), g("random_map_traffic_light_probability_weight", 1))
    s.features = list(g("features_to_include_in_observation", DEFAULT_FEATURES))
    s.sliding = bool(g("use_sliding_observation_window", False))
    s.sliding_size = int(g("sliding_observation_window_size", 4))
    s.next_subgoal = bool(g("use_next_subgoal_direction", False))
    s.sum_subgoals_reward = g("sum_subgoals_reward", 100)
    s.final_goal_bonus = g("final_goal_bonus", 0)
    s.crash_penalty = g("crash_penalty", 100)
    s.tl_violation_penalty = g("traffic_light_violation_penalty", 50)
    s.standing_still_penalty = g("standing_still_penalty", 0)
    s.visited_penalty = g("already_visited_position_penalty", 0)
    s.ice_probability = float(g("ice_probability", 0.1))
    s.street_damage_probability = float(g("street_damage_probability", 0.1))
    s.sand_probability = float(g("sand_probability", 0.2))
    s.traffic_density = float(g("traffic_density", 0.0))
    s.phase_dur = tuple(int(v) for v in g("traffic_light_phases_duration", (10, 3, 10)))
    s.ignore_traffic_collisions = bool(g("ignore_traffic_collisions", False))
    s.max_allowed_deviation = g("max_allowed_deviation", 10)
    s.profile_pct = (g("conservative_driver_percentage", 0.25), g("normal_driver_percentage", 0.35),
                     g("aggressive_driver_percentage", 0.20), g("elderly_driver_percentage", 0.15),
                     g("reckless_driver_percentage", 0.05))
    s.separate_reward_cost = bool(g("separate_reward_cost", False))
    s.render_mode = g("render_mode", None)
    s.map_path = map_path
    s.channels = feature_channels(s.features)
    if len(s.channels) > MAX_CHANNELS:
        raise ValueError(f"at most {MAX_CHANNELS} observation channels are supported")
    s.rules = [compile_rule(r) for r in DEFAULT_RULES]
    if s.render_mode not in (None, "human", "rgb_array", "pil_image"):
        raise Exception("the selected render_mode is not supported")

    if sum(s.phase_dur) <= 0:
        raise ZeroDivisionError("integer modulo by zero (traffic_light_phases_duration sums to 0)")

    # configuration warnings, pgtg/environment.py:366-412
    feats = s.features
    if s.obstacle_probability > 0:
        for wgt, name, msg in [
            (s.weights[0], "ice", "The ice obstacle"), (s.weights[1], "broken road", "The broken road obstacle"),
            (s.weights[2], "sand", "The sand obstacle")]:
            if wgt > 0 and name not in feats:
                warnings.warn(f"{msg} is used in the map generation but not included in the observation. "
                              "An agent will not be able to learn to avoid it.")
        for col in ("green", "yellow", "red"):
            if s.weights[3] > 0 and f"traffic_light_{col}" not in feats:
                warnings.warn(f"The traffic light obstacle is used in the map generation but {col} traffic "
                              "lights are not included in the observation. An agent will not be able to learn "
                              "to avoid it.")
    if s.traffic_density > 0 and "traffic" not in feats:
        warnings.warn("Traffic is generated but not included in the observation. An agent will not be able to "
                      "learn to avoid it.")

    if map_path is not None:
        s.fixed_map = json_file_to_map_plan(map_path)
    else:
        w, h = s.width, s.height
        sp = g("random_map_start_position", (0, -1, "west"))
        gp = g("random_map_goal_position", (-1, 0, "east"))
        s.start_mode, *sxyd = _parse_position(sp, "start_position", w, h)
        s.goal_mode, *gxyd = _parse_position(gp, "goal_position", w, h)
        s.start_xyd, s.goal_xyd = tuple(sxyd), tuple(gxyd)
        if s.start_mode == 0 and s.goal_mode == 0 and tuple(sp) == tuple(gp):
            raise ValueError("start_position and goal_position can't be the same tile and direction.")
        md = g("random_map_minimum_distance_between_start_and_goal", None)
        if md is not None and sp != "random" and gp != "random":
            raise ValueError("minimum_distance_between_start_and_goal can only be used if start_position and "
                             "goal_position are 'random'.")
        if md is not None and md > w + h - 2:
            raise ValueError("minimum_distance_between_start_and_goal can't be larger than width + height - 2.")
        s.min_distance = -1 if md is None else int(md)
        if s.obstacle_probability > 0 and sum(s.weights) == 0:
            raise ZeroDivisionError("float division by zero (all obstacle probability weights are 0)")
    return s


def add_rule(spec: EnvSpec, rule_dict: dict[str, Any]) -> None:
    """TrafficRuleEngine.add_rule (pgtg/environment.py:169-176)."""
    if any(r.name == rule_dict["name"] for r in spec.rules):
        raise ValueError(f"Rule with name {rule_dict['name']} already exists.")
    if len(spec.rules) >= MAX_RULES:
        raise ValueError(f"at most {MAX_RULES} traffic rules are supported")
    spec.rules.append(compile_rule(rule_dict))


def remove_rule(spec: EnvSpec, name: str) -> bool:
    for i, r in enumerate(spec.rules):
        if r.name == name:
            del spec.rules[i]
            return True
    return False
