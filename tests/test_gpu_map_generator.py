"""Procedural maps against the restatement, map by map: generate_map (pgtg/map_generator.py:43-189)
with its edge-removal loop (:192-266), which the kernel decides on the dual wall graph for maps of at
least 2 x 2 tiles and on the tile graph otherwise.  Every map size from 2 x 2 to 8 x 8
plus 1-wide strips and a w + h > 31 strip (the tile-graph fallback), under fixed, 2-tuple and random
start/goal positions (corner tiles, side tiles, start == goal tile) and connection percentages
0 .. 1: the tile exits, obstacles, start and goal of every sampled env's map after a seeded reset
and after the auto-resets of a short random rollout (the map-queue path) equal the restatement's."""
import itertools
import warnings

import numpy as np
import pytest

import helpers  # noqa: F401
from oracle.oracle import OracleEnv
from pgtg_amd import config as cfg

pytestmark = pytest.mark.gpu


def _positions(w, h, r):
    """start/goal kwargs: defaults, random, fixed border tuples (3- and 2-tuples), same tile"""
    side = [(0, int(r.integers(0, h)), "west"), (w - 1, int(r.integers(0, h)), "east"),
            (int(r.integers(0, w)), 0, "north"), (int(r.integers(0, w)), h - 1, "south")]
    a, b = side[int(r.integers(0, 4))], side[int(r.integers(0, 4))]
    out = [{}, dict(random_map_start_position="random", random_map_goal_position="random")]
    if a != b:
        out.append(dict(random_map_start_position=a, random_map_goal_position=b))
    if a[:2] != b[:2]:  # (the same tile with one possible direction would redraw forever, as in the reference)
        out.append(dict(random_map_start_position=a[:2], random_map_goal_position=b[:2]))
    t = side[0]
    same = (t[0], t[1], "west"), (t[0], t[1], "south" if t[1] == h - 1 else "north" if t[1] == 0 else "west")
    if same[0] != same[1]:
        out.append(dict(random_map_start_position=same[0], random_map_goal_position=same[1]))
    return out


def _cases():
    r = np.random.default_rng(5)
    sizes = list(itertools.product(range(2, 9), range(2, 9))) + [(1, 5), (6, 1), (2, 30), (31, 2)]
    out = []
    for w, h in sizes:
        for pos in _positions(w, h, r):
            pct = float(r.choice([0.0, 0.3, 0.5, 0.5, 0.85, 1.0]))
            out.append((w, h, pct, pos))
    return out


CASES = _cases()


def _spec(w, h, pct, pos, obst):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return cfg.make_spec(random_map_width=w, random_map_height=h, random_map_percentage_of_connections=pct,
                             random_map_obstacle_probability=obst, **pos)


def run_case(k: int) -> list:
    """maps of case k that differ from the restatement's (sampled envs, after the reset and after T steps)"""
    from pgtg_amd.vector import PGTGVecEnv
    w, h, pct, pos = CASES[k]
    n, sample, T = 128, 24, 6
    obst = 0.3 if k % 3 == 0 else 0.0
    try:
        spec = _spec(w, h, pct, pos, obst)
    except ValueError:
        return []  # a start/goal the reference rejects (tests/test_config.py)
    bad = []
    env = PGTGVecEnv(n, spec=spec, device=0)
    try:
        env.reset(seed=1000 * k)
        idx = np.random.default_rng(k).choice(n, sample, replace=False)
        orcs = {}
        for i in idx:
            o = OracleEnv(spec)
            o.reset(1000 * k + int(i))
            orcs[int(i)] = o
            if env.map_plan(int(i)) != o.map_plan():
                bad.append(f"case {k} {w}x{h} p={pct} {pos} env {int(i)} after reset")
        # auto-resets: the next episodes' maps (map queue or in-place resets)
        acts_dev = env.random_actions(T, 31 + k)
        acts = acts_dev.cpu().numpy()
        for t in range(T):
            env.step_actions(acts_dev[t])
            for i in idx:
                res = orcs[int(i)].step(int(acts[t, int(i)]))
                if res["terminated"]:
                    orcs[int(i)].reset(None)
        for i in idx:
            if env.map_plan(int(i)) != orcs[int(i)].map_plan():
                bad.append(f"case {k} {w}x{h} p={pct} {pos} env {int(i)} after {T} steps")
    finally:
        env.close()
    return bad


@pytest.mark.timeout(600)
def test_maps_every_size_and_start_goal():
    bad = []
    for k in range(len(CASES)):
        bad += run_case(k)
        if k % 25 == 0:
            print(f"map cases {k + 1}/{len(CASES)}", flush=True)
    cases = sorted({b.split(" env ")[0] for b in bad})
    assert not bad, f"{len(bad)} maps differ in {len(cases)} cases: {cases}; first: {bad[:3]}"


if __name__ == "__main__":  # one case: python tests/test_gpu_map_generator.py <k>
    import sys
    print(sys.argv[1], CASES[int(sys.argv[1])], run_case(int(sys.argv[1]))[:2], flush=True)
