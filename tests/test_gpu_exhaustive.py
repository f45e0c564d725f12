"""Exhaustive parity at the bench sizes: EVERY env of the batch, at EVERY step, against the CPU
restatement.  Both sides condense each env's step outputs (observation, terminal observation,
position, velocity, reward, termination, next-subgoal direction, cost) into the digest of
pgtg_amd/digest.py (the oracle computes the same formula in C, tests/test_digest.py pins the two
formulas to each other), so whole batches are compared without copying them to the host.

  configs[1]  4 096 envs x 100 steps, 3x3 maps                    (SURVEY.md 8(d) cfg 2)
  configs[3]  262 144 envs x 20 steps, 3x3 maps, in-kernel resets
  configs[4]  1 048 576 envs x 40 steps, 5x5 maps (the bench line; grid indexing past 2^20 envs; the
              map-queue rings through their refill steady state: a ring holds 3 episodes, a
              workgroup's helper wave refills <= 64 of them per launch)
  configs[4]'s 8-GPU shard 131 072 envs x 40 steps (one round of workgroups: the overflow lists)
  configs[2]  65 536 envs x 200 steps, 5x5 maps, traffic 0.5, with every env's car list in the
              digest (id, square, route, profile, patience, delay of every car after every step: the
              persisted occupancy counters, packing ticks, patience past patience_level*10), plus
              256 envs x 120 steps of cautious driving with the car lists compared (patience,
              crowded squares, spawner lists beyond the staged first 24)
  feature variants at batch sizes of every launch shape, incl. forced workgroup/sub-batch shapes.
"""
import warnings

import numpy as np
import pytest
import torch

import helpers  # noqa: F401
from oracle import oracle
from oracle.oracle import OracleEnv
from pgtg_amd import config as cfg

pytestmark = pytest.mark.gpu

ACT_SEED = 0xA11CE


def _spec(kw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return cfg.make_spec(**kw)


def _gpu_digests(spec, n, T, tune=None):
    from pgtg_amd.digest import Digest
    from pgtg_amd.vector import PGTGVecEnv
    env = PGTGVecEnv(n, spec=spec, device=0, tune=tune)
    try:
        env.reset(seed=0)
        dg = Digest(env)
        out = np.zeros((T, n), dtype=np.uint64)
        for t in range(T):
            env.step_random(ACT_SEED, t)
            out[t] = dg.step_digest().cpu().numpy().view(np.uint64)
        return out, env.step_kernel(), env.launch_info(), env.queue_overflow()
    finally:
        env.close()


def _compare(spec, n, T, tune=None, tag="", min_distinct=1000):
    got, kern, shape, ovf = _gpu_digests(spec, n, T, tune)
    ref = oracle.rollout_digest(spec, n, T, ACT_SEED)
    # the comparison has teeth: the rollout visits many distinct outputs.  Observations are local
    # 9x9 windows, so envs on small maps share digests (3x3 maps: 4 096 envs x 100 steps give 7 326
    # distinct ones, 262 144 x 20 give 13 072)
    assert len(np.unique(ref)) >= min(ref.size // 4, min_distinct), "degenerate digests"
    bad = np.argwhere(got != ref)
    assert bad.size == 0, (f"{tag} {kern} {shape}: {len(bad)} (step, env) digests differ, first {bad[:8].tolist()}")
    return ovf


# every feature name of the reference's vocabulary (pgtg/environment.py:1387-1445) plus names it does
# not know (all-zero channels): 61 observation keys
ALL_FEATURES = (["walls", "goals", "traffic", "traffic_light"] + list(cfg._GENERIC) +
                [f"unknown feature {k}" for k in range(14)])

CASES = {
    # name: (envs, steps, kwargs, launch-shape overrides)
    "cfg2_all_4096x100": (4096, 100, dict(random_map_width=3, random_map_height=3), None),
    "cfg4_all_262144x20": (262144, 20, dict(random_map_width=3, random_map_height=3), None),
    "cfg5_all_1048576x40": (1048576, 40, dict(random_map_width=5, random_map_height=5), None),
    "cfg3_all_65536x200": (65536, 200, dict(random_map_width=5, random_map_height=5, traffic_density=0.5), None),
    # feature variants over the launch shapes (16/32/64/128/256 envs per workgroup, sub-batched images)
    "obstacles_40000": (40000, 15, dict(random_map_width=4, random_map_height=4, random_map_obstacle_probability=1.0,
                                        random_map_ice_probability_weight=1, random_map_broken_road_probability_weight=1,
                                        random_map_sand_probability_weight=1,
                                        random_map_traffic_light_probability_weight=1, standing_still_penalty=0.5,
                                        already_visited_position_penalty=0.25, traffic_light_violation_penalty=2.0,
                                        separate_reward_cost=True), None),
    "sliding_nsd_12000": (12000, 15, dict(random_map_width=6, random_map_height=5, use_sliding_observation_window=True,
                                          sliding_observation_window_size=3, use_next_subgoal_direction=True), None),
    "features_140000": (140000, 12, dict(random_map_width=3, random_map_height=3,
                                         features_to_include_in_observation=["walls", "goals", "car_spawner",
                                                                             "car_lane all right", "traffic_light",
                                                                             "ice", "start", "final goal"],
                                         random_map_obstacle_probability=0.5), None),
    "sliding_traffic_6000": (6000, 8, dict(random_map_width=5, random_map_height=5, use_sliding_observation_window=True,
                                           sliding_observation_window_size=4, use_next_subgoal_direction=True,
                                           traffic_density=0.2), None),
    "features_all_names_3000": (3000, 10, dict(random_map_width=4, random_map_height=4, traffic_density=0.3,
                                               random_map_obstacle_probability=0.5,
                                               features_to_include_in_observation=ALL_FEATURES), None),
    # the reference's training caller (pgtg/train.py:21-37; bench.py --workload train): obstacles,
    # traffic with its driver mix, sliding window 5 and the next-subgoal direction together
    "train_caller_8192x30": (8192, 30, dict(random_map_width=4, random_map_height=4, random_map_obstacle_probability=0.2,
                                            random_map_percentage_of_connections=0.8, traffic_density=0.2,
                                            conservative_driver_percentage=0.15, normal_driver_percentage=0.50,
                                            aggressive_driver_percentage=0.20, elderly_driver_percentage=0.10,
                                            reckless_driver_percentage=0.05, sliding_observation_window_size=5,
                                            max_allowed_deviation=15, use_sliding_observation_window=True,
                                            use_next_subgoal_direction=True, final_goal_bonus=200,
                                            standing_still_penalty=1), None),
    # the map-queue step kernels at the shard sizes of 8 and 4 GPUs: k_envb (the automatic choice for
    # <= 2 rounds of workgroups: rings of three refilled per block) and configs[1] through k_envq's
    # persistent grid (tune_queue_mode 1)
    "cfg5_block_131072x40": (131072, 40, dict(random_map_width=5, random_map_height=5), None),
    "cfg5_block_262144x30": (262144, 30, dict(random_map_width=5, random_map_height=5), None),
    "cfg2_persistent_4096x100": (4096, 100, dict(random_map_width=3, random_map_height=3), dict(queue_mode=1)),
    "cfg2_wg256_sub32": (4096, 40, dict(random_map_width=3, random_map_height=3),
                         dict(envs_per_block=256, obs_sub=32)),
    "cfg5_wg256": (65536, 20, dict(random_map_width=5, random_map_height=5), dict(envs_per_block=256)),
    "cfg5_wg64": (20000, 20, dict(random_map_width=5, random_map_height=5), dict(envs_per_block=64)),
    # map queue with three env waves (192 envs per workgroup, two ring refills per helper lane), past
    # the rings' first turnover (40 steps) and with a ragged last workgroup
    "cfg5_wg192": (100000, 40, dict(random_map_width=5, random_map_height=5), dict(envs_per_block=192)),
    "cfg2_wg192": (30000, 40, dict(random_map_width=3, random_map_height=4), dict(envs_per_block=192)),
    "obstacles_wg32_sub8": (3000, 20, dict(random_map_width=4, random_map_height=4, random_map_obstacle_probability=1.0,
                                           standing_still_penalty=1.0), dict(envs_per_block=32, obs_sub=8)),
}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", sorted(CASES))
def test_every_env_every_step(name):
    n, T, kw, tune = CASES[name]
    _compare(_spec(kw), n, T, tune, name)


@pytest.mark.timeout(600)
def test_one_round_shard_overflow_path():
    """configs[4]'s per-GPU shard at N = 8 (131 072 envs: one round of map-queue workgroups) through
    k_envq's persistent grid (tune_queue_mode 1; the automatic choice there is k_envb, cfg5_block_*),
    every env at every step.  In a one-round launch a k_envq workgroup lists at most 64 ring-refill
    requests; the rest go to the overflow lists that other workgroups' helpers serve in the next launch.
    The device counter of overflow requests served shows that this path ran in the compared rollout."""
    ovf = _compare(_spec(dict(random_map_width=5, random_map_height=5)), 131072, 40, dict(queue_mode=1),
                   "cfg5_all_131072x40 (k_envq)")
    assert ovf > 0, "no overflow request was served: the one-round overflow path did not run"


@pytest.mark.timeout(600)
def test_cfg3_long_cautious_traffic():
    """configs[2] batch, 256 envs spread over the workgroups, 120 steps of mostly idle driving so that
    the episodes last and the traffic evolves: cars build patience past patience_level*10, squares
    crowd, despawned cars respawn from the whole spawner list.  Every step: observation, reward,
    termination; every 4th step and the last: the full car list (id, x, y, route, profile,
    patience, delay)."""
    from pgtg_amd.vector import PGTGVecEnv
    spec = _spec(dict(random_map_width=5, random_map_height=5, traffic_density=0.5))
    n, T = 65536, 120
    rng = np.random.default_rng(2024)
    idx = np.unique(np.concatenate([[0, 1, 63, 64, 127, 128, n // 2, n - 1], rng.choice(n, 248, replace=False)]))
    tix = torch.as_tensor(idx, device="cuda")
    env = PGTGVecEnv(n, spec=spec, device=0)
    try:
        env.reset(seed=77)
        orcs = {int(i): OracleEnv(spec) for i in idx}
        for i in idx:
            orcs[int(i)].reset(77 + int(i))
        max_pat, max_cars = 0, 0
        for t in range(T):
            acts = np.where(rng.random(n) < 0.9, 4, rng.integers(0, 9, n)).astype(np.uint8)
            env.step(torch.as_tensor(acts, device="cuda"))
            torch.cuda.synchronize()
            m = env.obs_map.index_select(0, tix).cpu().numpy()
            rew = env.reward.index_select(0, tix).cpu().numpy()
            term = env.terminated.index_select(0, tix).cpu().numpy()
            check_cars = t % 4 == 3 or t == T - 1
            for j, i in enumerate(idx):
                o = orcs[int(i)]
                r = o.step(int(acts[i]))
                tag = f"t{t} env{int(i)}"
                assert rew[j] == r["reward"] and bool(term[j]) == r["terminated"], tag + " reward/terminated"
                if r["terminated"]:
                    r = o.reset(None)
                assert np.array_equal(m[j], r["obs"]), tag + " obs"
                if check_cars:
                    oc = o.cars()
                    assert np.array_equal(env.cars(int(i)), oc), tag + " cars"
                    if len(oc):
                        max_pat = max(max_pat, int(oc[:, 5].max()))
                        max_cars = max(max_cars, len(oc))
        # the long horizon did reach the regimes it is meant to cover
        assert max_pat > 10, max_pat
        assert max_cars > 200, max_cars
    finally:
        env.close()
