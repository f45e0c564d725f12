"""Host-side pieces of the single-env facade (no GPU): the compass used for
info['traffic_rules']['agent_direction'], and loud failure without the HIP device."""
import math

import numpy as np
import pytest

from pgtg_amd.env import SQ_FINAL_GOAL, SQ_SUBGOAL, compass_direction


def _reference_compass(goal, x, y, window):
    """pgtg/environment.py:1037-1090 restated literally (nested loops, strict <, atan2 octants)."""
    best, dmin = None, float("inf")
    W, H = goal.shape
    for tx in range(W):
        for ty in range(H):
            if goal[tx, ty]:
                d = abs(tx - x) + abs(ty - y)
                if d < dmin:
                    dmin, best = d, (tx, ty)
    if best is None:
        return -1
    dx, dy = best[0] - x, best[1] - y
    if abs(dx) <= window and abs(dy) <= window:
        return -1
    a = math.atan2(dy, dx)
    p8 = math.pi / 8
    table = [(-p8, p8, 2), (p8, 3 * p8, 3), (3 * p8, 5 * p8, 4), (5 * p8, 7 * p8, 5),
             (-7 * p8, -5 * p8, 7), (-5 * p8, -3 * p8, 0), (-3 * p8, -p8, 1)]
    for lo, hi, k in table:
        if lo <= a < hi:
            return k
    return 6


@pytest.mark.parametrize("seed", range(40))
def test_compass_matches_reference_restatement(seed):
    rng = np.random.default_rng(seed)
    W, H = 9 * int(rng.integers(1, 6)), 9 * int(rng.integers(1, 6))
    goal = rng.random((W, H)) < rng.choice([0.0, 0.002, 0.01, 0.05])
    sq = np.zeros((W, H), np.uint64)
    sq[goal] |= np.uint64(SQ_SUBGOAL if seed % 2 else SQ_FINAL_GOAL)
    sq |= np.uint64(1 << 32) * (rng.random((W, H)) < 0.3).astype(np.uint64)  # walls do not matter
    for _ in range(20):
        x, y = int(rng.integers(-2, W + 2)), int(rng.integers(-2, H + 2))
        window = int(rng.integers(0, 6))
        assert compass_direction(sq, x, y, window) == _reference_compass(goal, x, y, window)


def test_facade_needs_the_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by test_gpu_env.py")
    from pgtg_amd.env import PGTGEnv
    with pytest.raises((RuntimeError, AssertionError)):
        PGTGEnv(random_map_width=3, random_map_height=3)


def test_unknown_render_mode_rejected_before_device_use():
    """environment.py:790 accepts None/human/rgb_array/pil_image and raises for anything else; this
    happens in the config, before any device use."""
    from pgtg_amd.env import PGTGEnv
    with pytest.raises(Exception, match="render_mode"):
        PGTGEnv(render_mode="svg")
