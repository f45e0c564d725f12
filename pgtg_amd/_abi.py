"""ctypes mirror of include/pgtg.h and the loader of the in-tree HIP library.

The product path has no CPU fallback: if `libpgtg_hip.so` is missing or cannot be loaded, every
entry point raises.  (The CPU oracle under oracle/ is test infrastructure and is never used here.)
"""
from __future__ import annotations

import ctypes as C
import os

from . import config as cfgmod

PKG = os.path.dirname(os.path.abspath(__file__))
# PGTG_LIB selects another build of the same library (test variants, pgtg_amd/build.py VARIANTS)
LIB_PATH = os.environ.get("PGTG_LIB") or os.path.join(PKG, "libpgtg_hip.so")

PGTG_ABI_VERSION = 7
MAX_TILES = 256
MAX_CHANNELS = 128
MAX_RULES = 8

PGTG_OK = 0
PGTG_E_INVALID = -1
PGTG_E_DONE = -2
PGTG_E_DEVICE = -3
PGTG_E_UNSUPPORTED = -4
PGTG_E_MAP = -5

EXPORTED = [
    "pgtg_create", "pgtg_destroy", "pgtg_set_stream", "pgtg_set_outputs", "pgtg_reset",
    "pgtg_reset_unseeded", "pgtg_step", "pgtg_step_many", "pgtg_random_actions", "pgtg_get_env_state", "pgtg_get_cars",
    "pgtg_get_map_plan", "pgtg_get_squares", "pgtg_set_rules", "pgtg_set_agent", "pgtg_add_car", "pgtg_observe", "pgtg_get_counters",
    "pgtg_error_count", "pgtg_window", "pgtg_num_envs", "pgtg_launch_info", "pgtg_occupancy", "pgtg_step_kernel", "pgtg_last_error", "pgtg_enable_timing",
    "pgtg_timing_read", "pgtg_measure_hbm", "pgtg_state_size", "pgtg_dump_state", "pgtg_load_state",
    "pgtg_set_to_state", "pgtg_car_digest", "pgtg_get_queue_maps", "pgtg_get_queue_overflow", "pgtg_set_flat_outputs", "pgtg_set_flat_scalars",
]


class PgtgRule(C.Structure):
    _fields_ = [("tile_exits", C.c_int32), ("speed_sq_min", C.c_int32), ("speed_sq_max", C.c_int32),
                ("min_traffic", C.c_int32), ("min_matching_traffic", C.c_int32),
                ("weight", (C.c_uint8 * 20) * 6)]


class PgtgConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("width", C.c_int32), ("height", C.c_int32),
        ("pct_connections", C.c_double), ("start_mode", C.c_int32), ("goal_mode", C.c_int32),
        ("start_x", C.c_int32), ("start_y", C.c_int32), ("start_dir", C.c_int32),
        ("goal_x", C.c_int32), ("goal_y", C.c_int32), ("goal_dir", C.c_int32),
        ("min_distance", C.c_int32), ("obstacle_probability", C.c_double),
        ("w_ice", C.c_double), ("w_broken", C.c_double), ("w_sand", C.c_double), ("w_tl", C.c_double),
        ("n_channels", C.c_int32), ("channels", C.c_int32 * MAX_CHANNELS),
        ("sliding", C.c_int32), ("sliding_size", C.c_int32), ("next_subgoal", C.c_int32),
        ("sum_subgoals_reward", C.c_double), ("final_goal_bonus", C.c_double),
        ("crash_penalty", C.c_double), ("tl_violation_penalty", C.c_double),
        ("standing_still_penalty", C.c_double), ("visited_penalty", C.c_double),
        ("ice_probability", C.c_double), ("street_damage_probability", C.c_double),
        ("sand_probability", C.c_double), ("traffic_density", C.c_double),
        ("phase_dur", C.c_int32 * 3), ("ignore_traffic_collisions", C.c_int32),
        ("profile_pct", C.c_double * 5), ("separate_reward_cost", C.c_int32),
        ("n_rules", C.c_int32), ("rules", PgtgRule * MAX_RULES),
        ("fixed_map", C.c_int32), ("fm_w", C.c_int32), ("fm_h", C.c_int32),
        ("fm_exits", C.c_uint8 * MAX_TILES), ("fm_obst_type", C.c_int8 * MAX_TILES),
        ("fm_obst_mask", C.c_int8 * MAX_TILES), ("fm_start", C.c_int32 * 3), ("fm_goal", C.c_int32 * 3),
        ("autoreset", C.c_int32), ("max_episode_steps", C.c_int32), ("min_car_capacity", C.c_int32),
        ("tune_envs_per_block", C.c_int32), ("tune_obs_sub", C.c_int32), ("tune_kt_grid", C.c_int32),
        ("tune_kt_cap", C.c_int32), ("tune_kt_wpc", C.c_int32), ("tune_car_slots", C.c_int32),
        ("tune_kt_serial", C.c_int32), ("tune_queue_mode", C.c_int32), ("tune_fault", C.c_int32),
    ]


class PgtgOutputs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "obs", "position", "velocity", "next_subgoal", "reward", "cost", "terminated", "truncated",
        "final_obs", "final_position", "final_velocity", "final_next_subgoal", "braking")]


class PgtgEnvState(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("x", "y", "vx", "vy", "terminated", "flat_tire", "phase", "elapsed",
                                         "n_cars", "next_car_id", "path_len", "error")] + [
        ("spawn_counter", C.c_uint32), ("seed", C.c_uint64), ("used_subgoals", C.c_uint64 * 4),
        ("n_spawners", C.c_int32), ("car_tail", C.c_int32)]


class PgtgCar(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("id", "x", "y", "route", "profile", "patience", "delay")]


_lib = None


def lib():
    """Load the in-tree HIP library (raises if it is missing: no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `python -m pgtg_amd.build` (HIP/gfx950); "
                           "there is no CPU fallback")
    # torch ships its own libamdhip64/libhsa-runtime64 (same soname as /opt/rocm's).  Load it first
    # so that this library binds to the process's single HIP runtime and shares torch's device
    # memory and streams; loading ours first would start a second HSA runtime.
    import torch  # noqa: F401
    L = C.CDLL(LIB_PATH)
    vp, u64, i32 = C.c_void_p, C.c_uint64, C.c_int32
    sig = {
        "pgtg_create": ([C.POINTER(PgtgConfig), u64, i32, C.POINTER(vp)], C.c_int),
        "pgtg_destroy": ([vp], C.c_int),
        "pgtg_set_stream": ([vp, vp], C.c_int),
        "pgtg_set_outputs": ([vp, C.POINTER(PgtgOutputs)], C.c_int),
        "pgtg_reset": ([vp, vp, u64, vp], C.c_int),
        "pgtg_reset_unseeded": ([vp, vp], C.c_int),
        "pgtg_step": ([vp, vp], C.c_int),
        "pgtg_step_many": ([vp, vp, u64, u64], C.c_int),
        "pgtg_random_actions": ([vp, vp, u64, u64, u64], C.c_int),
        "pgtg_measure_hbm": ([i32, u64, i32, C.POINTER(C.c_double)], C.c_int),
        "pgtg_state_size": ([vp, C.POINTER(u64)], C.c_int),
        "pgtg_dump_state": ([vp, vp, u64], C.c_int),
        "pgtg_load_state": ([vp, vp, u64], C.c_int),
        "pgtg_set_to_state": ([vp, u64, i32, i32, i32, i32, i32, C.POINTER(PgtgCar), i32], C.c_int),
        "pgtg_get_env_state": ([vp, u64, C.POINTER(PgtgEnvState)], C.c_int),
        "pgtg_get_cars": ([vp, u64, C.POINTER(PgtgCar), i32, C.POINTER(i32)], C.c_int),
        "pgtg_get_map_plan": ([vp, u64] + [vp] * 7, C.c_int),
        "pgtg_get_squares": ([vp, u64, vp, i32, C.POINTER(i32), C.POINTER(i32)], C.c_int),
        "pgtg_set_rules": ([vp, vp, i32], C.c_int),
        "pgtg_set_agent": ([vp, u64, i32, i32, i32, i32], C.c_int),
        "pgtg_add_car": ([vp, u64, i32, i32, i32, i32, i32], C.c_int),
        "pgtg_observe": ([vp], C.c_int),
        "pgtg_get_counters": ([vp, C.POINTER(u64), C.POINTER(u64)], C.c_int),
        "pgtg_car_digest": ([vp, vp], C.c_int),
        "pgtg_get_queue_maps": ([vp, C.POINTER(u64)], C.c_int),
        "pgtg_get_queue_overflow": ([vp, C.POINTER(u64)], C.c_int),
        "pgtg_set_flat_outputs": ([vp, C.POINTER(C.c_int32), i32, i32, vp, vp], C.c_int),
        "pgtg_set_flat_scalars": ([vp, vp, vp, vp], C.c_int),
        "pgtg_error_count": ([vp, C.POINTER(u64), C.POINTER(i32)], C.c_int),
        "pgtg_window": ([vp], C.c_int),
        "pgtg_num_envs": ([vp], u64),
        "pgtg_launch_info": ([vp, C.POINTER(i32), C.POINTER(i32)], C.c_int),
        "pgtg_occupancy": ([vp, C.POINTER(i32)], C.c_int),
        "pgtg_step_kernel": ([vp], C.c_char_p),
        "pgtg_last_error": ([vp], C.c_char_p),
        "pgtg_timing_read": ([vp, C.POINTER(C.c_double), C.POINTER(u64), i32], C.c_int),
        "pgtg_enable_timing": ([vp, i32], C.c_int),
    }
    # A/B runs against an older build of the library (tools/ab_multi.sh): PGTG_ABI_COMPAT names its ABI
    # version; entry points it does not have are left unbound
    compat = os.environ.get("PGTG_ABI_COMPAT")
    for name, (args, res) in sig.items():
        if compat and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def fill_rules(dst, rules) -> int:
    """Compiled traffic rules (config.CompiledRule) into a PgtgRule array; returns the count."""
    if len(rules) > MAX_RULES:
        raise ValueError(f"at most {MAX_RULES} traffic rules are supported")
    for i, r in enumerate(rules):
        o = dst[i]
        o.tile_exits, o.speed_sq_min, o.speed_sq_max = r.tile_exits, r.speed_sq_min, r.speed_sq_max
        o.min_traffic, o.min_matching_traffic = r.min_traffic, r.min_matching_traffic
        for d in range(6):
            for k in range(20):
                o.weight[d][k] = r.weight[d][k]
    return len(rules)


TUNE_KEYS = ("envs_per_block", "obs_sub", "kt_grid", "kt_cap", "kt_wpc", "car_slots", "kt_serial", "queue_mode", "fault")


def config_struct(spec: "cfgmod.EnvSpec", autoreset: bool, max_episode_steps: int | None,
                  min_car_capacity: int = 0, tune: dict | None = None) -> PgtgConfig:
    c = PgtgConfig()
    c.abi_version = int(os.environ.get("PGTG_ABI_COMPAT") or PGTG_ABI_VERSION)
    c.width, c.height = spec.width, spec.height
    c.pct_connections = spec.pct_connections
    c.start_mode, c.goal_mode = spec.start_mode, spec.goal_mode
    c.start_x, c.start_y, c.start_dir = spec.start_xyd
    c.goal_x, c.goal_y, c.goal_dir = spec.goal_xyd
    c.min_distance = spec.min_distance
    c.obstacle_probability = spec.obstacle_probability
    c.w_ice, c.w_broken, c.w_sand, c.w_tl = [float(w) for w in spec.weights]
    c.n_channels = len(spec.channels)
    for i, (_, code) in enumerate(spec.channels):
        c.channels[i] = code
    c.sliding, c.sliding_size, c.next_subgoal = int(spec.sliding), spec.sliding_size, int(spec.next_subgoal)
    c.sum_subgoals_reward = spec.sum_subgoals_reward
    c.final_goal_bonus = spec.final_goal_bonus
    c.crash_penalty = spec.crash_penalty
    c.tl_violation_penalty = spec.tl_violation_penalty
    c.standing_still_penalty = spec.standing_still_penalty
    c.visited_penalty = spec.visited_penalty
    c.ice_probability = spec.ice_probability
    c.street_damage_probability = spec.street_damage_probability
    c.sand_probability = spec.sand_probability
    c.traffic_density = spec.traffic_density
    for i in range(3):
        c.phase_dur[i] = spec.phase_dur[i]
    c.ignore_traffic_collisions = int(spec.ignore_traffic_collisions)
    for i in range(5):
        c.profile_pct[i] = float(spec.profile_pct[i])
    c.separate_reward_cost = int(spec.separate_reward_cost)
    c.n_rules = fill_rules(c.rules, spec.rules)
    fm = spec.fixed_map
    if fm is not None:
        if fm.width * fm.height > MAX_TILES:
            raise ValueError(f"this build supports maps of at most {MAX_TILES} tiles")
        c.fixed_map = 1
        c.fm_w, c.fm_h = fm.width, fm.height
        for i in range(fm.width * fm.height):
            c.fm_exits[i] = fm.exits[i]
            c.fm_obst_type[i] = fm.obstacle_type[i]
            c.fm_obst_mask[i] = fm.obstacle_mask[i]
        for i in range(3):
            c.fm_start[i] = fm.start[i]
            c.fm_goal[i] = fm.goal[i]
    c.autoreset = int(autoreset)
    c.max_episode_steps = int(max_episode_steps or 0)
    c.min_car_capacity = int(min_car_capacity)
    for k, v in (tune or {}).items():
        if k not in TUNE_KEYS:
            raise ValueError(f"unknown launch-shape override {k!r} (one of {TUNE_KEYS})")
        setattr(c, "tune_" + k, int(v))
    return c
