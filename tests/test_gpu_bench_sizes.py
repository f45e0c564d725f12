"""Parity at the bench sizes (BASELINE.json configs[1..4]): the golden replays run small batches,
which take the small-workgroup launch shapes; these run the full batches (the launch shapes the
bench measures: 128-env map-queue workgroups, 256-env workgroups, traffic workgroups) and compare a
sample of envs spread over workgroups, waves and lanes with the CPU oracle, every step, including
terminal observations and same-step auto-resets."""
import warnings

import numpy as np
import pytest
import torch

import helpers  # noqa: F401
from oracle.oracle import OracleEnv
from pgtg_amd import config as cfg

pytestmark = pytest.mark.gpu

CASES = {
    "cfg2": (4096, dict(random_map_width=3, random_map_height=3), 40),
    "cfg5": (131072, dict(random_map_width=5, random_map_height=5), 30),
    "cfg4": (262144, dict(random_map_width=3, random_map_height=3), 30),
    "cfg3": (65536, dict(random_map_width=5, random_map_height=5, traffic_density=0.5), 12),
    # feature variants at multi-workgroup scale (other launch shapes and code paths than the above):
    # obstacles with every RNG stream, penalties and the cost channel (the map queue with stream resets)
    "obstacles": (32768, dict(random_map_width=4, random_map_height=4, random_map_obstacle_probability=1.0,
                              random_map_ice_probability_weight=1, random_map_broken_road_probability_weight=1,
                              random_map_sand_probability_weight=1, random_map_traffic_light_probability_weight=1,
                              standing_still_penalty=0.5, already_visited_position_penalty=0.25,
                              traffic_light_violation_penalty=2.0, separate_reward_cost=True), 25),
    # sliding window + next-subgoal direction + light traffic (k_env<true> generic observation path,
    # k_traffic, the observe launch for windows other than the agent's tile)
    "sliding_traffic": (16384, dict(random_map_width=5, random_map_height=5, use_sliding_observation_window=True,
                                    sliding_observation_window_size=4, use_next_subgoal_direction=True,
                                    traffic_density=0.2), 12),
    # custom feature list (lanes, spawners, lights) on the fixed-tile window
    "features": (32768, dict(random_map_width=3, random_map_height=3,
                             features_to_include_in_observation=["walls", "goals", "car_spawner",
                                                                  "car_lane all right", "traffic_light", "ice"]), 25),
}


def _sample(n: int, k: int) -> np.ndarray:
    rng = np.random.default_rng(n)
    fixed = [0, 1, 63, 64, 127, 128, 191, 255, 256, n // 2, n - 129, n - 128, n - 65, n - 64, n - 1]
    return np.unique(np.concatenate([np.array(fixed), rng.choice(n, k - len(fixed), replace=False)]))


@pytest.mark.parametrize("name", sorted(CASES))
def test_bench_size_parity(name):
    from pgtg_amd.vector import PGTGVecEnv
    n, kw, T = CASES[name]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        spec = cfg.make_spec(**kw)
    idx = _sample(n, 24 if spec.traffic_density > 0 else 40)
    tix = torch.as_tensor(idx, device="cuda")
    env = PGTGVecEnv(n, spec=spec, device=0)
    try:
        env.reset(seed=7)
        orcs = {int(i): OracleEnv(spec) for i in idx}
        m0 = env.obs_map.index_select(0, tix).cpu().numpy()
        for j, i in enumerate(idx):
            r = orcs[int(i)].reset(7 + int(i))
            assert np.array_equal(m0[j], r["obs"]), f"{name} reset obs env {int(i)}"
        acts = env.random_actions(T, 0xA11CE)
        for t in range(T):
            env.step_actions(acts[t])
            torch.cuda.synchronize()
            a = acts[t].index_select(0, tix).cpu().numpy()
            m = env.obs_map.index_select(0, tix).cpu().numpy()
            fm = env.final_map.index_select(0, tix).cpu().numpy()
            rew = env.reward.index_select(0, tix).cpu().numpy()
            term = env.terminated.index_select(0, tix).cpu().numpy()
            pos = env.position.index_select(0, tix).cpu().numpy()
            cost = env.cost.index_select(0, tix).cpu().numpy() if env.cost is not None else None
            nsd = env.nsd.index_select(0, tix).cpu().numpy() if env.nsd is not None else None
            for j, i in enumerate(idx):
                o = orcs[int(i)]
                r = o.step(int(a[j]))
                tag = f"{name} t{t} env{int(i)}"
                assert rew[j] == r["reward"] and bool(term[j]) == r["terminated"], tag + " reward/terminated"
                if cost is not None:
                    assert cost[j] == r["cost"], tag + " cost"
                if r["terminated"]:
                    assert np.array_equal(fm[j], r["obs"]), tag + " terminal obs"
                    r = o.reset(None)
                assert np.array_equal(m[j], r["obs"]), tag + " obs"
                assert tuple(pos[j]) == tuple(r["pos"]), tag + " position"
                if nsd is not None:
                    assert int(nsd[j]) == int(r["nsd"]), tag + " next subgoal direction"
                if spec.traffic_density > 0:
                    assert np.array_equal(env.cars(int(i)), o.cars()), tag + " cars"
    finally:
        env.close()
