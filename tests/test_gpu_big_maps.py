"""Maps of more than 64 tiles (up to 16 x 16): the 256-bit generator / path compiler, the global edge
table, used subgoals kept in the plan words (kPlanUsed) and paths longer than 64 tiles.

  * the reference's own integration-test environment (tests/test_integration.py:25-50, a 9 x 9 map
    with obstacles, traffic and penalties) through the single-env facade: construct, reset, render,
    get_info, step(4), against the CPU restatement;
  * every env at every step (digest of pgtg_amd/digest.py, car lists included with traffic) against
    the restatement at 10 x 10, 12 x 12 and 16 x 16 and the launch shapes those batches pick.
The golden replays of tests/golden/traj_s9_integration / s10_obstacles / s16_traffic (made from the
reference by tools/gen_golden.py) run in test_gpu_parity.py."""
import warnings

import numpy as np
import pytest

import helpers  # noqa: F401
from oracle import oracle
from oracle.oracle import OracleEnv
from pgtg_amd import config as cfg

pytestmark = pytest.mark.gpu

ACT_SEED = 0xB16

# tests/test_integration.py:25-42 (test_complex_random_generated_map_environment)
INTEGRATION_KW = dict(random_map_width=9, random_map_height=9, random_map_percentage_of_connections=0.9,
                      random_map_obstacle_probability=0.8, random_map_broken_road_probability_weight=2,
                      random_map_ice_probability_weight=4, random_map_sand_probability_weight=8,
                      render_mode="pil_image", final_goal_bonus=100, standing_still_penalty=5,
                      ice_probability=0.5, street_damage_probability=0.2, traffic_density=0.02,
                      ignore_traffic_collisions=True)


def _spec(kw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return cfg.make_spec(**kw)


@pytest.mark.parametrize("seed", [0, 1, 7, 2024])
def test_reference_integration_environment(seed):
    from pgtg_amd.env import PGTGEnv
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        env = PGTGEnv(**INTEGRATION_KW)
    orc = OracleEnv(_spec(INTEGRATION_KW))
    try:
        obs, info = env.reset(seed=seed)
        r = orc.reset(seed)
        assert env.render() is None
        assert isinstance(env.get_info(), dict)
        keys = [k for k, _ in env.spec.channels]
        rng = np.random.default_rng(seed)
        for t in range(30):
            a = 4 if t == 0 else int(rng.integers(0, 9))
            obs, rew, term, trunc, info = env.step(a)
            env.render()
            env.get_info()
            r = orc.step(a)
            for c, k in enumerate(keys):
                assert np.array_equal(obs["map"][k], r["obs"][c].astype(np.int64)), f"t{t} {k}"
            assert tuple(obs["position"]) == tuple(r["pos"]) and tuple(obs["velocity"]) == tuple(r["vel"]), t
            assert rew == r["reward"] and term == r["terminated"], t
            assert np.array_equal(env._vec.cars(0), orc.cars()), f"t{t} cars"
            if term:
                break
    finally:
        env.close()


def _digests(spec, n, T):
    from pgtg_amd.digest import Digest
    from pgtg_amd.vector import PGTGVecEnv
    env = PGTGVecEnv(n, spec=spec, device=0)
    try:
        env.reset(seed=0)
        dg = Digest(env)
        out = np.zeros((T, n), dtype=np.uint64)
        for t in range(T):
            env.step_random(ACT_SEED, t)
            out[t] = dg.step_digest().cpu().numpy().view(np.uint64)
        return out, env.step_kernel(), env.launch_info()
    finally:
        env.close()


CASES = {
    # name: (envs, steps, kwargs)
    "s10_obstacles_6000x15": (6000, 15, dict(random_map_width=10, random_map_height=10,
                                             random_map_obstacle_probability=0.6, standing_still_penalty=1,
                                             already_visited_position_penalty=0.5, use_next_subgoal_direction=True)),
    "s12_queue_40000x8": (40000, 8, dict(random_map_width=12, random_map_height=12,
                                         random_map_percentage_of_connections=0.3)),
    "s16_full_3000x8": (3000, 8, dict(random_map_width=16, random_map_height=16,
                                      random_map_percentage_of_connections=0.95)),
    "s16x4_strip_5000x10": (5000, 10, dict(random_map_width=16, random_map_height=5,
                                           random_map_percentage_of_connections=0.2)),
    "s9_traffic_3000x10": (3000, 10, dict(random_map_width=9, random_map_height=9, traffic_density=0.3)),
    "s11_sliding_2000x10": (2000, 10, dict(random_map_width=11, random_map_height=9,
                                           use_sliding_observation_window=True, sliding_observation_window_size=10,
                                           use_next_subgoal_direction=True)),
}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", sorted(CASES))
def test_big_maps_every_env_every_step(name):
    n, T, kw = CASES[name]
    spec = _spec(kw)
    got, kern, shape = _digests(spec, n, T)
    ref = oracle.rollout_digest(spec, n, T, ACT_SEED)
    bad = np.argwhere(got != ref)
    assert bad.size == 0, f"{name} {kern} {shape}: {len(bad)} (step, env) digests differ, first {bad[:8].tolist()}"
    assert "true>" in kern or "true," in kern, kern  # the > 64-tile kernel instance ran


def test_long_paths_reward_share():
    """Random maps rarely have shortest paths beyond 64 tiles; a snake-like fixed 9 x 9 map forces one
    through all 81 tiles: the subgoal reward share sum/81 (DevCfg::ind_reward beyond the LDS table)."""
    import json
    import os
    import tempfile
    from pgtg_amd.env import PGTGEnv
    w, h = 9, 9
    # boustrophedon path through all 81 tiles, row by row: east along even rows, west along odd rows
    tiles = [[{"exits": [0, 0, 0, 0]} for _ in range(w)] for _ in range(h)]

    def link(x0, y0, x1, y1):
        d = {(1, 0): (1, 3), (-1, 0): (3, 1), (0, 1): (2, 0), (0, -1): (0, 2)}[(x1 - x0, y1 - y0)]
        tiles[y0][x0]["exits"][d[0]] = 1
        tiles[y1][x1]["exits"][d[1]] = 1

    order = [(x if y % 2 == 0 else w - 1 - x, y) for y in range(h) for x in range(w)]
    for (x0, y0), (x1, y1) in zip(order, order[1:]):
        link(x0, y0, x1, y1)
    tiles[0][0]["exits"][3] = 1  # start: west border of (0, 0)
    gx = order[-1][0]  # row 8 runs east: the path ends at (8, 8), leaving through its east border
    tiles[h - 1][gx]["exits"][1] = 1
    plan = {"width": w, "height": h, "map": tiles, "start": [0, 0, "west"], "goal": [gx, h - 1, "east"]}
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "snake.json")
        json.dump(plan, open(p, "w"))
        env = PGTGEnv(p, sum_subgoals_reward=1000)
        spec = cfg.make_spec(p, sum_subgoals_reward=1000)
        orc = OracleEnv(spec)
        try:
            env.reset(seed=3)
            orc.reset(3)
            assert env._vec.env_state(0)["path_len"] == 81
            total = 0.0
            for t in range(60):  # accelerate east along row 0: the subgoals of tiles 0..7, then the wall
                _, rew, term, _, _ = env.step(7)
                r = orc.step(7)
                assert rew == r["reward"] and term == r["terminated"], t
                total += max(rew, 0.0)
                if term:
                    break
            assert total >= 4 * 1000 / 81, total  # several shares of sum/81 were paid
        finally:
            env.close()
