"""Container-only: generate golden vectors by running the REFERENCE (imported through the
stand-ins of tools/refshim, see tools/refload.py) and write them as small compressed fixtures to
tests/golden/.  The reference itself never travels; only these data files do.

Vector semantics (what the batched product implements): env i is reset with seed `seed_base+i`,
then stepped with actions[t, i]; when it terminates it is reset unseeded (next spawn block), the
gymnasium/SB3 auto-reset convention.  Recorded per (t, i): the step's returned observation
(terminal one when it ended), reward, cost, terminated, position, velocity, next_subgoal_direction,
a digest of the car list, and the post-reset observation of envs that were reset.

Usage:  python tools/gen_golden.py [name ...]
"""
import json
import os
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import refload  # noqa: E402

env_mod, mg, rparser, rmap, td, const = refload.load()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "tests", "golden")
TESTDATA = "/root/reference/tests/test_data"
ROUTES = sorted({f.split()[1] for t in td.TRAFFIC_LANES.values() for c in t for s in c for f in s
                 if f.startswith("car_lane") and f.split()[1] != "all"})
PROFILES = ["conservative", "normal", "aggressive", "elderly", "reckless"]
# obstacle mask ids: constants.OBSTACLE_MASK_NAMES order, then the traffic-light masks
OMASKS = list(const.OBSTACLE_MASK_NAMES) + [m for m in td.OBSTACLE_MASKS if m.startswith("traffic_light")]

CONFIGS = {
    # name: (kwargs, map_path, n_envs, steps, action_mode)
    "s3_default": (dict(random_map_width=3, random_map_height=3), None, 48, 100, "uniform"),
    "s3_obstacles": (dict(random_map_width=3, random_map_height=3, random_map_obstacle_probability=1.0),
                     None, 32, 60, "cautious"),
    "s3_obstacles_tlkey": (dict(random_map_width=3, random_map_height=3, random_map_obstacle_probability=0.7,
                                random_map_traffic_light_probability_weight=3,
                                features_to_include_in_observation=["walls", "goals", "traffic_light", "sand",
                                                                    "start", "used subgoal", "car_spawner",
                                                                    "car_lane all right", "nonexistent"]),
                           None, 16, 60, "cautious"),
    "s5_default": (dict(random_map_width=5, random_map_height=5), None, 24, 60, "uniform"),
    "s5_traffic05": (dict(random_map_width=5, random_map_height=5, traffic_density=0.5), None, 6, 40, "cautious"),
    "s4_train": (dict(random_map_width=4, random_map_height=4, random_map_obstacle_probability=0.2,
                      traffic_density=0.2, use_sliding_observation_window=True,
                      sliding_observation_window_size=5, use_next_subgoal_direction=True),
                 None, 12, 60, "cautious"),
    "s4_penalties": (dict(traffic_density=0.1, ignore_traffic_collisions=True, standing_still_penalty=3,
                          already_visited_position_penalty=2, final_goal_bonus=7, separate_reward_cost=True),
                     None, 12, 60, "cautious"),
    "s4_nsd_fixed": (dict(use_next_subgoal_direction=True, random_map_obstacle_probability=0.3,
                          sum_subgoals_reward=7), None, 16, 50, "uniform"),
    "tl_heavy": (dict(random_map_width=3, random_map_height=3, random_map_obstacle_probability=1.0,
                      random_map_traffic_light_probability_weight=1000, traffic_density=0.3,
                      traffic_light_phases_duration=(2, 1, 2), features_to_include_in_observation=[
                          "walls", "goals", "traffic", "traffic_light"]),
                 None, 8, 60, "cautious"),
    "random_start_goal": (dict(random_map_width=4, random_map_height=3, random_map_start_position="random",
                               random_map_goal_position="random",
                               random_map_minimum_distance_between_start_and_goal=3,
                               random_map_obstacle_probability=0.3), None, 24, 40, "uniform"),
    "start_goal_2tuple": (dict(random_map_width=3, random_map_height=4, random_map_start_position=(0, 2),
                               random_map_goal_position=(-1, -1), random_map_percentage_of_connections=0.8),
                          None, 16, 40, "uniform"),
    "tiny_1x1": (dict(random_map_width=1, random_map_height=1, traffic_density=0.5), None, 8, 30, "uniform"),
    "strip_2x1_full": (dict(random_map_width=2, random_map_height=1, random_map_percentage_of_connections=1.0),
                       None, 8, 30, "uniform"),
    # maps of > 64 tiles (the 256-bit generator path): the reference's own integration-test env
    # (tests/test_integration.py:25-42, 9x9), a 10x10 with obstacles and penalties, a 16x16 with traffic
    "s9_integration": (dict(random_map_width=9, random_map_height=9, random_map_percentage_of_connections=0.9,
                            random_map_obstacle_probability=0.8, random_map_broken_road_probability_weight=2,
                            random_map_ice_probability_weight=4, random_map_sand_probability_weight=8,
                            render_mode="pil_image", final_goal_bonus=100, standing_still_penalty=5,
                            ice_probability=0.5, street_damage_probability=0.2, traffic_density=0.02,
                            ignore_traffic_collisions=True), None, 8, 40, "uniform"),
    "s10_obstacles": (dict(random_map_width=10, random_map_height=10, random_map_obstacle_probability=0.5,
                           use_next_subgoal_direction=True, already_visited_position_penalty=1,
                           separate_reward_cost=True), None, 6, 50, "cautious"),
    "s16_traffic": (dict(random_map_width=16, random_map_height=16, random_map_percentage_of_connections=0.7,
                         traffic_density=0.1, use_sliding_observation_window=True,
                         sliding_observation_window_size=6), None, 3, 30, "cautious"),
    "fixed_1x1_traffic": (dict(traffic_density=1, ignore_traffic_collisions=True), "1x1_map", 4, 40, "still"),
    "fixed_crossing": (dict(traffic_density=0.5), "1x1_crossing_map", 4, 40, "cautious"),
    "fixed_4x1": (dict(sum_subgoals_reward=444), "4x1_map.json", 4, 40, "cautious"),
    "fixed_deadends": (dict(traffic_density=0.3, ignore_traffic_collisions=True), "map_with_all_deadends",
                       3, 30, "cautious"),
}


def actions_for(mode, T, N, seed):
    rng = np.random.default_rng(seed)
    if mode == "uniform":
        return rng.integers(0, 9, size=(T, N)).astype(np.uint8)
    if mode == "still":
        return np.full((T, N), 4, np.uint8)
    # cautious: mostly coast, sometimes accelerate, keeps episodes alive for many ticks
    a = rng.integers(0, 9, size=(T, N)).astype(np.uint8)
    keep = rng.random((T, N)) < 0.6
    a[keep] = 4
    return a


def car_rows(env):
    return np.array([[c.id, c.position.x, c.position.y, ROUTES.index(c.route), PROFILES.index(c.driver_profile.value),
                      c.patience_counter, int(c.last_action_delay)] for c in env.cars], dtype=np.int32).reshape(-1, 7)


def digest(arr):
    return zlib.crc32(np.ascontiguousarray(arr, dtype=np.int32).tobytes())


def obs_stack(obs, keys):
    return np.stack([np.asarray(obs["map"][k], dtype=np.uint8) for k in keys])


def plan_rows(env):
    mp = env.map_plan
    ex, ot, om = [], [], []
    for y in range(mp.height):
        for x in range(mp.width):
            t = mp.tiles[y][x]
            ex.append(sum(int(b) << i for i, b in enumerate(t["exits"])))
            ot.append(const.OBSTACLE_NAMES.index(t["obstacle_type"]) if t.get("obstacle_type") else -1)
            om.append(OMASKS.index(t["obstacle_mask"]) if t.get("obstacle_mask") else -1)
    dirs = ["north", "east", "south", "west"]
    return dict(w=mp.width, h=mp.height, exits=ex, otype=ot, omask=om,
                start=[int(mp.start[0]), int(mp.start[1]), dirs.index(mp.start[2])],
                goal=[int(mp.goal[0]), int(mp.goal[1]), dirs.index(mp.goal[2])])


def run(name):
    kwargs, map_file, N, T, mode = CONFIGS[name]
    map_path = os.path.join(TESTDATA, map_file) if map_file else None
    seed_base = 0
    acts = actions_for(mode, T, N, 12345)
    cwd = os.getcwd()
    os.chdir(REPO)
    envs = [env_mod.PGTGEnv(map_path, **kwargs) for _ in range(N)]
    os.chdir(cwd)
    first = [e.reset(seed=seed_base + i)[0] for i, e in enumerate(envs)]
    keys = list(first[0]["map"].keys())
    W = np.asarray(first[0]["map"][keys[0]]).shape[0]
    C = len(keys)
    init_obs = np.stack([obs_stack(o, keys) for o in first])
    init_pos = np.array([o["position"] for o in first], np.int32)
    init_nsd = np.array([o.get("next_subgoal_direction", -1) for o in first], np.int32)
    obs = np.zeros((T, N, C, W, W), np.uint8)
    pos = np.zeros((T, N, 2), np.int32)
    vel = np.zeros((T, N, 2), np.int32)
    rew = np.zeros((T, N), np.float64)
    cost = np.zeros((T, N), np.float64)
    term = np.zeros((T, N), np.uint8)
    nsd = np.zeros((T, N), np.int32)
    brake = np.zeros((T, N), np.uint8)
    cars_dig = np.zeros((T, N), np.uint32)
    ncars = np.zeros((T, N), np.int32)
    reset_obs, reset_idx, reset_pos, reset_nsd, reset_dig = [], [], [], [], []
    plans = [[plan_rows(e)] for e in envs]
    init_cars = [car_rows(e) for e in envs]
    cars_final = []
    for t in range(T):
        for i, e in enumerate(envs):
            o, r, te, tr, info = e.step(int(acts[t, i]))
            obs[t, i] = obs_stack(o, keys)
            pos[t, i] = o["position"]
            vel[t, i] = o["velocity"]
            rew[t, i] = float(r)
            cost[t, i] = float(info.get("cost", 0))
            term[t, i] = bool(te)
            nsd[t, i] = o.get("next_subgoal_direction", -1)
            brake[t, i] = bool(e.braking_applied)
            cr = car_rows(e)
            cars_dig[t, i] = digest(cr)
            ncars[t, i] = len(cr)
            if te:
                o2, _ = e.reset()
                reset_obs.append(obs_stack(o2, keys))
                reset_idx.append((t, i))
                reset_pos.append(o2["position"])
                reset_nsd.append(o2.get("next_subgoal_direction", -1))
                reset_dig.append(digest(car_rows(e)))
                plans[i].append(plan_rows(e))
    for e in envs:
        cars_final.append(car_rows(e))
    meta = dict(name=name, kwargs=kwargs, map_file=map_file, N=N, T=T, seed_base=seed_base, keys=keys,
                action_mode=mode, plans=plans)
    R = len(reset_idx)
    np.savez_compressed(
        os.path.join(OUT, f"traj_{name}.npz"),
        meta=np.frombuffer(json.dumps(meta).encode(), np.uint8), actions=acts,
        init_obs=init_obs, init_pos=init_pos, init_nsd=init_nsd,
        init_cars_dig=np.array([digest(c) for c in init_cars], np.uint32),
        obs=obs, pos=pos, vel=vel, reward=rew, cost=cost, terminated=term, nsd=nsd, braking=brake,
        cars_dig=cars_dig, ncars=ncars,
        reset_idx=np.array(reset_idx, np.int32).reshape(R, 2),
        reset_obs=np.array(reset_obs, np.uint8).reshape(R, C, W, W),
        reset_pos=np.array(reset_pos, np.int32).reshape(R, 2),
        reset_nsd=np.array(reset_nsd, np.int32).reshape(R),
        reset_cars_dig=np.array(reset_dig, np.uint32).reshape(R),
        cars_final=np.concatenate(cars_final) if cars_final else np.zeros((0, 7), np.int32),
        cars_final_n=np.array([len(c) for c in cars_final], np.int32),
    )
    return R, int(term.sum())


def reproducibility_fixture():
    """The reference's own golden trajectory (tests/test_data/reproducibility_data.py) as data."""
    import importlib.util
    sp = importlib.util.spec_from_file_location("repro", os.path.join(TESTDATA, "reproducibility_data.py"))
    m = importlib.util.module_from_spec(sp)
    sp.loader.exec_module(m)
    fx = m.COMPLICATED_ENVIRONMENT
    keys = list(fx["observation_list"][0]["map"].keys())
    obs = np.stack([obs_stack(o, keys) for o in fx["observation_list"]])
    np.savez_compressed(
        os.path.join(OUT, "ref_complicated_environment.npz"),
        meta=np.frombuffer(json.dumps(dict(kwargs=fx["environment_arguments"], seed=fx["seed"], keys=keys)).encode(),
                           np.uint8),
        actions=np.array(fx["action_list"], np.int32), obs=obs,
        pos=np.array([o["position"] for o in fx["observation_list"]], np.int32),
        vel=np.array([o["velocity"] for o in fx["observation_list"]], np.int32),
        reward=np.array(fx["reward_list"], np.float64),
        terminated=np.array(fx["terminated_list"], np.uint8),
        truncated=np.array(fx["truncated_list"], np.uint8))


def rng_vectors():
    """numpy Generator known answers for the restated primitives (numpy 2.2.6 here; locked 1.26.4)."""
    out = {}
    seeds = np.array([0, 1, 7, 123456789, 2**32 + 5, 2**63 + 11], np.uint64)
    keys = np.array([0, 1, 4, 5, 9, 1000], np.uint32)
    st = np.zeros((len(seeds), len(keys), 4), np.uint64)
    raw = np.zeros((len(seeds), len(keys), 8), np.uint64)
    for a, s in enumerate(seeds):
        for b, k in enumerate(keys):
            g = np.random.PCG64(np.random.SeedSequence(int(s), spawn_key=(int(k),)))
            sd = g.state["state"]
            st[a, b] = [sd["state"] >> 64, sd["state"] & (2**64 - 1), sd["inc"] >> 64, sd["inc"] & (2**64 - 1)]
            raw[a, b] = g.random_raw(8)
    out["seeds"], out["keys"], out["pcg_state"], out["pcg_raw"] = seeds, keys, st, raw
    # mixed draw script on one stream
    g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(42, spawn_key=(3,))))
    script, vals = [], []
    prng = np.random.default_rng(7)
    for t in range(2000):
        kind = int(prng.integers(0, 4))
        if kind == 0:
            script.append((0, 0)); vals.append(g.random())
        elif kind == 1:
            n = int(prng.integers(1, 3000)); script.append((1, n)); vals.append(float(g.integers(0, n)))
        elif kind == 2:
            script.append((2, 0)); vals.append(float(g.choice(5, p=[0.25, 0.35, 0.2, 0.15, 0.05])))
        else:
            script.append((3, 0)); vals.append(float(g.integers(1, 4)))
    out["script"] = np.array(script, np.int64)
    out["script_vals"] = np.array(vals, np.float64)
    g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(9, spawn_key=(1,))))
    nr = []
    for pop, k in [(10, 3), (474, 237), (18, 18), (5, 1), (2025, 1012), (1, 1), (729, 100)]:
        nr.append(np.array([pop, k] + list(g.choice(pop, size=k, replace=False)), np.int64))
    out["noreplace"] = np.concatenate(nr)
    np.savez_compressed(os.path.join(OUT, "rng_numpy.npz"), **out)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    names = sys.argv[1:] or list(CONFIGS)
    if not sys.argv[1:]:
        rng_vectors()
        reproducibility_fixture()
    for n in names:
        import time
        t0 = time.time()
        R, nt = run(n)
        print(f"{n}: resets={R} terminations={nt} {time.time() - t0:.1f}s", flush=True)
