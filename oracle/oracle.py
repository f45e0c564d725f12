"""ctypes binding of the CPU oracle (oracle/pgtg_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker / the timed CPU baseline; the product (pgtg_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

MAX_FEATURES = 128
MAX_RULES = 8


class OrcRule(C.Structure):
    _fields_ = [("tile_exits", C.c_int32), ("vel_lo", C.c_double), ("vel_hi", C.c_double),
                ("min_traffic", C.c_int32), ("min_matching_traffic", C.c_int32),
                ("weight", (C.c_uint8 * 20) * 6)]


class OrcConfig(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("pct_connections", C.c_double),
        ("start_mode", C.c_int32), ("goal_mode", C.c_int32),
        ("start_x", C.c_int32), ("start_y", C.c_int32), ("start_dir", C.c_int32),
        ("goal_x", C.c_int32), ("goal_y", C.c_int32), ("goal_dir", C.c_int32),
        ("min_distance", C.c_int32), ("obstacle_probability", C.c_double),
        ("w_ice", C.c_double), ("w_broken", C.c_double), ("w_sand", C.c_double), ("w_tl", C.c_double),
        ("n_channels", C.c_int32), ("channels", C.c_int32 * MAX_FEATURES),
        ("sliding", C.c_int32), ("sliding_size", C.c_int32), ("next_subgoal", C.c_int32),
        ("sum_subgoals_reward", C.c_double), ("final_goal_bonus", C.c_double),
        ("crash_penalty", C.c_double), ("tl_violation_penalty", C.c_double),
        ("standing_still_penalty", C.c_double), ("visited_penalty", C.c_double),
        ("ice_probability", C.c_double), ("street_damage_probability", C.c_double),
        ("sand_probability", C.c_double), ("traffic_density", C.c_double),
        ("phase_dur", C.c_int32 * 3), ("ignore_traffic_collisions", C.c_int32),
        ("profile_pct", C.c_double * 5), ("separate_reward_cost", C.c_int32),
        ("n_rules", C.c_int32), ("rules", OrcRule * MAX_RULES),
        ("fixed_map", C.c_int32), ("fm_w", C.c_int32), ("fm_h", C.c_int32),
        ("fm_exits", C.c_uint8 * 1024), ("fm_obst_type", C.c_int8 * 1024),
        ("fm_obst_mask", C.c_int8 * 1024), ("fm_start", C.c_int32 * 3), ("fm_goal", C.c_int32 * 3),
    ]


class OrcOut(C.Structure):
    _fields_ = [("pos", C.c_int32 * 2), ("vel", C.c_int32 * 2), ("reward", C.c_double),
                ("cost", C.c_double), ("terminated", C.c_int32), ("truncated", C.c_int32),
                ("next_subgoal_direction", C.c_int32), ("braking", C.c_int32)]


class OrcCar(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("id", "x", "y", "route", "profile", "patience", "delay")]


class OrcPcg(C.Structure):
    _fields_ = [("st_hi", C.c_uint64), ("st_lo", C.c_uint64), ("inc_hi", C.c_uint64),
                ("inc_lo", C.c_uint64), ("has32", C.c_int32), ("buf32", C.c_uint32)]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_create.restype = C.c_void_p
        L.orc_create.argtypes = [C.POINTER(OrcConfig)]
        L.orc_destroy.argtypes = [C.c_void_p]
        L.orc_reset.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.POINTER(OrcOut)]
        L.orc_step.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.POINTER(OrcOut)]
        L.orc_window.argtypes = [C.c_void_p]
        L.orc_num_cars.argtypes = [C.c_void_p]
        L.orc_get_cars.argtypes = [C.c_void_p, C.POINTER(OrcCar), C.c_int]
        L.orc_get_map_plan.argtypes = [C.c_void_p] + [C.c_void_p] * 7
        L.orc_get_misc.argtypes = [C.c_void_p] + [C.c_void_p] * 4
        L.orc_set_agent.argtypes = [C.c_void_p] + [C.c_int32] * 4
        L.orc_add_car.argtypes = [C.c_void_p] + [C.c_int32] * 5
        L.orc_get_squares.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.orc_set_to_state.argtypes = [C.c_void_p] + [C.c_int32] * 5 + [C.POINTER(OrcCar), C.c_int32, C.c_void_p,
                                                                         C.POINTER(OrcOut)]
        L.orc_last_error.restype = C.c_char_p
        L.orc_last_error.argtypes = [C.c_void_p]
        L.orc_seed_seq_state.argtypes = [C.POINTER(C.c_uint32), C.c_int, C.POINTER(C.c_uint32)]
        L.orc_pcg64_from_seed.argtypes = [C.c_uint64, C.c_uint32, C.c_int, C.POINTER(OrcPcg)]
        L.orc_next64.restype = C.c_uint64
        L.orc_next64.argtypes = [C.POINTER(OrcPcg)]
        L.orc_next32.restype = C.c_uint32
        L.orc_next32.argtypes = [C.POINTER(OrcPcg)]
        L.orc_random.restype = C.c_double
        L.orc_random.argtypes = [C.POINTER(OrcPcg)]
        L.orc_integers.restype = C.c_int64
        L.orc_integers.argtypes = [C.POINTER(OrcPcg), C.c_int64, C.c_int64]
        L.orc_choice_p.restype = C.c_int64
        L.orc_choice_p.argtypes = [C.POINTER(OrcPcg), C.POINTER(C.c_double), C.c_int]
        L.orc_choice_noreplace.argtypes = [C.POINTER(OrcPcg), C.c_int64, C.c_int64, C.POINTER(C.c_int64)]
        L.orc_bench.restype = C.c_int64
        L.orc_bench.argtypes = [C.POINTER(OrcConfig), C.c_int, C.c_int, C.c_uint64, C.c_uint64]
        L.orc_rollout_digest.restype = C.c_int
        L.orc_rollout_digest.argtypes = [C.POINTER(OrcConfig), C.c_int64, C.c_uint64, C.c_int, C.c_uint64, C.c_void_p]
        _lib = L
    return _lib


def config_from_spec(spec) -> OrcConfig:
    c = OrcConfig()
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
    c.n_rules = len(spec.rules)
    for i, r in enumerate(spec.rules):
        o = c.rules[i]
        o.tile_exits, o.vel_lo, o.vel_hi = r.tile_exits, r.vel_lo, r.vel_hi
        o.min_traffic, o.min_matching_traffic = r.min_traffic, r.min_matching_traffic
        for d in range(6):
            for k in range(20):
                o.weight[d][k] = r.weight[d][k]
    fm = spec.fixed_map
    if fm is not None:
        c.fixed_map = 1
        c.fm_w, c.fm_h = fm.width, fm.height
        for i in range(fm.width * fm.height):
            c.fm_exits[i] = fm.exits[i]
            c.fm_obst_type[i] = fm.obstacle_type[i]
            c.fm_obst_mask[i] = fm.obstacle_mask[i]
        for i in range(3):
            c.fm_start[i] = fm.start[i]
            c.fm_goal[i] = fm.goal[i]
    return c


def bench(spec, n_envs: int, steps: int, seed_base: int = 0, act_seed: int = 12345) -> int:
    """Run the oracle's built-in random-action rollout loop (bench.py cpu_baseline); env-steps done."""
    c = config_from_spec(spec)
    n = lib().orc_bench(C.byref(c), int(n_envs), int(steps), int(seed_base), int(act_seed))
    if n < 0:
        raise RuntimeError("oracle bench failed")
    return n


def host_threads() -> int:
    """Host cores this process may use (the GPU box's CPU share is 16, whatever os.cpu_count() says)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16
    return max(1, min(n, cap))


def _parallel(fn, n_envs: int, threads: int, chunk_min: int = 256):
    """Run fn(lo, hi) over [0, n_envs) in `threads` host threads (ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    lib()
    threads = max(1, min(threads, (n_envs + chunk_min - 1) // chunk_min))
    bounds = [(n_envs * k // threads, n_envs * (k + 1) // threads) for k in range(threads)]
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(lambda b: fn(*b), bounds))


def rollout_digest(spec, n_envs: int, steps: int, act_seed: int, env_offset: int = 0, threads: int = 0) -> np.ndarray:
    """[steps, n_envs] uint64 output digests of global envs env_offset..+n_envs (seed = global index,
    actions = the GPU's splitmix hash), the formula of pgtg_amd/digest.py."""
    c = config_from_spec(spec)
    out = np.zeros((steps, n_envs), dtype=np.uint64)
    # warm the library's one-time tables on this thread before fanning out
    e = lib().orc_create(C.byref(c))
    lib().orc_destroy(e)

    def run(lo, hi):
        if hi <= lo:
            return 0
        part = np.zeros((steps, hi - lo), dtype=np.uint64)
        rc = lib().orc_rollout_digest(C.byref(c), hi - lo, env_offset + lo, steps, act_seed, part.ctypes.data)
        if rc:
            raise RuntimeError("oracle rollout failed")
        out[:, lo:hi] = part
        return hi - lo

    _parallel(run, n_envs, threads or host_threads())
    return out


def bench_parallel(spec, n_envs: int, steps: int, threads: int, act_seed: int = 12345) -> int:
    """orc_bench over `threads` host threads (disjoint env ranges); env-steps done."""
    c = config_from_spec(spec)
    e = lib().orc_create(C.byref(c))
    lib().orc_destroy(e)

    def run(lo, hi):
        if hi <= lo:
            return 0
        n = lib().orc_bench(C.byref(c), hi - lo, steps, lo, act_seed)
        if n < 0:
            raise RuntimeError("oracle bench failed")
        return n

    return sum(_parallel(run, n_envs, threads, chunk_min=1))


class OracleEnv:
    """Single reference-semantics environment on the CPU oracle (test/baseline use only)."""

    def __init__(self, spec):
        self.spec = spec
        self._cfg = config_from_spec(spec)
        self._L = lib()
        self._h = self._L.orc_create(C.byref(self._cfg))
        self.win = self._L.orc_window(self._h)
        self.nch = len(spec.channels)
        self.obs = np.zeros((self.nch, self.win, self.win), np.uint8)
        self.out = OrcOut()

    def __del__(self):
        try:
            self._L.orc_destroy(self._h)
        except Exception:
            pass

    def _err(self):
        return self._L.orc_last_error(self._h).decode()

    def reset(self, seed: int | None = None):
        rc = self._L.orc_reset(self._h, -1 if seed is None else int(seed), self.obs.ctypes.data, C.byref(self.out))
        if rc:
            raise RuntimeError(self._err())
        return self.result()

    def step(self, action: int):
        rc = self._L.orc_step(self._h, int(action), self.obs.ctypes.data, C.byref(self.out))
        if rc:
            msg = self._err()
            raise RuntimeError(msg)
        return self.result()

    def result(self) -> dict:
        o = self.out
        return {"obs": self.obs.copy(), "pos": (o.pos[0], o.pos[1]), "vel": (o.vel[0], o.vel[1]),
                "reward": o.reward, "cost": o.cost, "terminated": bool(o.terminated),
                "truncated": bool(o.truncated), "nsd": o.next_subgoal_direction, "braking": o.braking}

    def cars(self) -> np.ndarray:
        n = self._L.orc_num_cars(self._h)
        arr = (OrcCar * max(n, 1))()
        self._L.orc_get_cars(self._h, arr, n)
        return np.array([[c.id, c.x, c.y, c.route, c.profile, c.patience, c.delay] for c in arr[:n]],
                        dtype=np.int32).reshape(n, 7)

    def map_plan(self):
        w, h = C.c_int32(), C.c_int32()
        ex = (C.c_uint8 * 1024)()
        ot = (C.c_int8 * 1024)()
        om = (C.c_int8 * 1024)()
        s3 = (C.c_int32 * 3)()
        g3 = (C.c_int32 * 3)()
        self._L.orc_get_map_plan(self._h, C.byref(w), C.byref(h), ex, ot, om, s3, g3)
        n = w.value * h.value
        return {"w": w.value, "h": h.value, "exits": list(ex[:n]), "otype": list(ot[:n]),
                "omask": list(om[:n]), "start": tuple(s3), "goal": tuple(g3)}

    def misc(self):
        ph, ft, nid = C.c_int32(), C.c_int32(), C.c_int32()
        sc = C.c_uint32()
        self._L.orc_get_misc(self._h, C.byref(ph), C.byref(ft), C.byref(nid), C.byref(sc))
        return {"phase": ph.value, "flat_tire": ft.value, "next_car_id": nid.value, "spawn_counter": sc.value}

    def set_agent(self, x, y, vx=None, vy=None):
        o = self.out
        self._L.orc_set_agent(self._h, int(x), int(y), int(o.vel[0] if vx is None else vx),
                              int(o.vel[1] if vy is None else vy))

    def add_car(self, x, y, route: int, profile: int, car_id: int = -1):
        self._L.orc_add_car(self._h, int(x), int(y), int(route), int(profile), int(car_id))

    def set_to_state(self, x, y, vx, vy, flat_tire, cars=()):
        """PGTGEnv.set_to_state; cars = [(id, x, y, route, profile)]; returns the observation result."""
        cars = list(cars)
        arr = (OrcCar * max(1, len(cars)))()
        for k, (cid, cx, cy, route, prof) in enumerate(cars):
            arr[k].id, arr[k].x, arr[k].y, arr[k].route, arr[k].profile = cid, cx, cy, route, prof
        self._L.orc_set_to_state(self._h, int(x), int(y), int(vx), int(vy), int(bool(flat_tire)), arr, len(cars),
                                 self.obs.ctypes.data, C.byref(self.out))
        return self.result()

    def squares(self) -> np.ndarray:
        n = self._L.orc_get_squares(self._h, None, 0)
        out = np.zeros(n, np.uint64)
        self._L.orc_get_squares(self._h, out.ctypes.data, n)
        return out
