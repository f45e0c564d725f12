"""Velocity decomposition at large speeds on the GPU (pgtg/environment.py:693-748, _round :29-30).

Random-action episodes rarely exceed |v| = 3, so here every velocity with |vx|, |vy| <= 64 is set
directly (set_to_state) on an 8x8-tile map of crossings and stepped once with zero acceleration, from
two start squares.  Each env is compared with the CPU oracle put into the same state (observation,
position, reward, termination), and its resting square with the reference decomposition restated
in numpy (tests/decompose_ref.py, pinned to the reference's known answers): the agent stops on the
first sub-step square that is a wall or off the map, else at p0 + v.  This reaches the |dx| = 10 and
|dx| = 22 cases where a fused multiply-add or integer arithmetic would round differently."""
import json

import numpy as np
import pytest
import torch

import decompose_ref as dr
import helpers  # noqa: F401
from oracle.oracle import OracleEnv
from pgtg_amd import config as cfg

pytestmark = pytest.mark.gpu

V = 64
STARTS = [(31, 31), (36, 31)]  # centre of tile (3,3); west exit segment of tile (4,3)
SQ_WALL = np.uint64(1 << 32)
SQ_FINAL = np.uint64(1 << 41)


def _crossing_map(path, n=8):
    tiles = [[{"exits": [1, 1, 1, 1]} for _ in range(n)] for _ in range(n)]
    json.dump({"width": n, "height": n, "map": tiles, "start": [0, 0, "west"], "goal": [n - 1, n - 1, "east"]},
              open(path, "w"))


@pytest.mark.timeout(600)
def test_every_velocity_up_to_64(tmp_path):
    from pgtg_amd.vector import PGTGVecEnv
    mp = str(tmp_path / "crossings.json")
    _crossing_map(mp)
    spec = cfg.make_spec(mp)
    vels = [(vx, vy) for vx in range(-V, V + 1) for vy in range(-V, V + 1)]
    cases = [(s, v) for s in STARTS for v in vels]
    n = len(cases)
    env = PGTGVecEnv(n, spec=spec, device=0, autoreset=False)
    orc = OracleEnv(spec)
    try:
        env.reset(seed=5)
        for i, ((x, y), (vx, vy)) in enumerate(cases):
            env.set_to_state(i, x, y, vx, vy, False)
        env.step(torch.full((n,), 4, dtype=torch.uint8, device="cuda"))
        torch.cuda.synchronize()
        obs, pos = env.obs_map.cpu().numpy(), env.position.cpu().numpy()
        rew, term = env.reward.cpu().numpy(), env.terminated.cpu().numpy()
        sq = None
        independent = 0
        for i, ((x, y), (vx, vy)) in enumerate(cases):
            orc.reset(5 + i)
            orc.set_to_state(x, y, vx, vy, False)
            r = orc.step(4)
            tag = f"start {(x, y)} v {(vx, vy)}"
            assert rew[i] == r["reward"] and bool(term[i]) == r["terminated"], tag + " reward/terminated"
            assert tuple(pos[i]) == tuple(r["pos"]), tag + f" position {tuple(pos[i])} vs oracle {r['pos']}"
            assert np.array_equal(obs[i], r["obs"]), tag + " observation"
            if sq is None:
                sq = orc.squares().reshape(72, 72)
            # independent: walk the restated decomposition
            cx, cy, stop, goal = x, y, None, False
            for px, py in dr.decompose(vx, vy):
                cx, cy = cx + px, cy + py
                if not (0 <= cx < 72 and 0 <= cy < 72) or (sq[cx, cy] & SQ_WALL):
                    stop = (cx, cy)
                    break
                if sq[cx, cy] & SQ_FINAL:
                    goal = True
                    break
            if goal:
                continue
            ex, ey = stop if stop is not None else (x + vx, y + vy)
            # observation position: the square clamped into the map, relative to its tile
            # (environment.py:1352-1366, 1446-1460)
            cx_, cy_ = min(max(ex, 0), 71), min(max(ey, 0), 71)
            assert tuple(pos[i]) == (cx_ % 9, cy_ % 9), tag + f" rests at {(ex, ey)} by the reference decomposition"
            assert bool(term[i]) == (stop is not None), tag + " crash"
            independent += 1
        assert independent > 0.9 * n
    finally:
        env.close()
