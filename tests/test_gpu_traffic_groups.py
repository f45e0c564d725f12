"""k_traffic's launch shapes against the CPU oracle: the work list is levelled over the grid's waves
(`e` envs per wave, in rounds beyond the LDS capacity `cap`) and each env gets min(16, 64 / e) lanes
(pgtg_env.hip k_traffic / traffic_reset).  The launch-shape overrides tune_kt_grid / tune_kt_cap force every
shape with small batches: 16, 12, 8, 4, 3 and 2 lanes per env, one env per wave in many rounds.  The per-car draws
of the initial traffic run lane-parallel (cars_group: each lane jumps the env's car stream to its
cars); tune_kt_serial forces the one-lane loop that a Lemire rejection falls back to."""

import numpy as np
import pytest
import torch

import helpers  # noqa: F401
from oracle.oracle import OracleEnv
from pgtg_amd import config as cfg

pytestmark = pytest.mark.gpu

# (envs, grid, cap, map w x h): the initial reset puts every env on the work list, so
# e = ceil(n / (4 * grid))
SHAPES = {
    "quads_e16": (512, 8, None, (5, 5)),     # e = 16 -> 4 lanes per env
    "triples_e20": (640, 8, None, (5, 5)),   # e = 20 -> 3 lanes
    "pairs_e25": (800, 8, None, (5, 5)),     # e = 25 -> 2 lanes
    "g16_e3": (96, 8, None, (5, 5)),         # e = 3 -> 16 lanes per env (the steady configs[2] shape)
    "g8_e8": (256, 8, None, (5, 5)),         # e = 8 -> 8 lanes
    "g12_e5": (160, 8, None, (5, 5)),        # e = 5 -> 12 lanes (a group that is no power of two)
    "rounds_cap1": (96, 4, 1, (5, 5)),       # e = 1, six rounds per wave, 16 lanes per env
    "rounds_cap5": (700, 4, 5, (5, 5)),      # e = 5 in nine rounds of the 16 waves, 12 lanes per env
    # more than seven tile rows: the lookup's per-tile row search instead of the column row masks
    "tall_map": (256, 8, None, (2, 9)),
    "wide_map": (256, 8, None, (9, 2)),
    # the per-car draws on one lane per env (the rejection fallback of cars_group)
    "serial_quads_e16": (512, 8, None, (5, 5), {"kt_serial": 1}),
    "serial_pairs_e25": (800, 8, None, (5, 5), {"kt_serial": 1}),
    "serial_g16_e3": (96, 8, None, (5, 5), {"kt_serial": 1}),
}


@pytest.mark.parametrize("name", sorted(SHAPES))
def test_traffic_launch_shapes(name):
    from pgtg_amd.vector import PGTGVecEnv
    n, grid, cap, (mw, mh), *extra = SHAPES[name]
    spec = cfg.make_spec(random_map_width=mw, random_map_height=mh, traffic_density=0.5)
    tune = {"kt_grid": grid} if cap is None else {"kt_grid": grid, "kt_cap": cap}
    if extra:
        tune.update(extra[0])
    env = PGTGVecEnv(n, spec=spec, device=0, tune=tune)
    rng = np.random.default_rng(n)
    idx = np.unique(np.concatenate([[0, 1, 2, n // 2, n - 2, n - 1], rng.choice(n, 12, replace=False)]))
    tix = torch.as_tensor(idx, device="cuda")
    try:
        env.reset(seed=11)
        orcs = {int(i): OracleEnv(spec) for i in idx}
        m0 = env.obs_map.index_select(0, tix).cpu().numpy()
        for j, i in enumerate(idx):
            r = orcs[int(i)].reset(11 + int(i))
            assert np.array_equal(m0[j], r["obs"]), f"{name} reset obs env {int(i)}"
            assert np.array_equal(env.cars(int(i)), orcs[int(i)].cars()), f"{name} reset cars env {int(i)}"
        acts = env.random_actions(8, 0xBEE)
        for t in range(8):
            env.step_actions(acts[t])
            torch.cuda.synchronize()
            a = acts[t].index_select(0, tix).cpu().numpy()
            m = env.obs_map.index_select(0, tix).cpu().numpy()
            rew = env.reward.index_select(0, tix).cpu().numpy()
            term = env.terminated.index_select(0, tix).cpu().numpy()
            for j, i in enumerate(idx):
                o = orcs[int(i)]
                r = o.step(int(a[j]))
                tag = f"{name} t{t} env{int(i)}"
                assert rew[j] == r["reward"] and bool(term[j]) == r["terminated"], tag + " reward/terminated"
                if r["terminated"]:
                    r = o.reset(None)
                assert np.array_equal(m[j], r["obs"]), tag + " obs"
                assert np.array_equal(env.cars(int(i)), o.cars()), tag + " cars"
    finally:
        env.close()
