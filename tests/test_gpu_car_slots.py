"""The single-bank car store (pgtg_amd/csrc/pgtg_env.hip move_cars): survivors are rewritten in
place, a despawned car leaves an empty slot, respawns are appended behind the tail, and a wave in
which some env starts a tick with more than 4 empty slots packs its lists (survivors to packed slots
with their ids, respawns moved down behind them).  The list order the reference keeps
(`for car in copy.copy(self.cars)` / `self.cars.remove(car)` / `self.cars.append(...)`,
pgtg/environment.py:1121-1127) must survive all of it.

Long cautious episodes (the agent mostly idles, so episodes last and cars keep respawning, so
packing ticks come every few ticks) on the smallest slot budget the library accepts (3 x capacity +
4) are compared with the CPU restatement at every step (observation, reward, termination) and the
full car lists (id, x, y, route, profile, patience, delay) every third step.  The same rollout runs
again through the build whose occupancy counters saturate at 2 cars (exact recounts from the slots
on nearly every car move)."""
import os
import subprocess
import sys
import warnings

import numpy as np
import pytest

import helpers  # noqa: F401

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cautious_rollout(width, height, density, n, steps, n_sample, seed, slots_extra=0):
    """Returns (mismatches, compactions seen, max tail, max cars)."""
    import torch
    from oracle.oracle import OracleEnv
    from pgtg_amd import config as cfg
    from pgtg_amd.vector import PGTGVecEnv
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        spec = cfg.make_spec(random_map_width=width, random_map_height=height, traffic_density=density)
    cap = int(width * height * 32 * density)
    env = PGTGVecEnv(n, spec=spec, device=0, tune={"car_slots": 3 * cap + 4 + slots_extra})
    bad, compactions, max_tail, max_cars = [], 0, 0, 0
    try:
        env.reset(seed=seed)
        rng = np.random.default_rng(seed)
        idx = np.unique(np.concatenate([[0, 1, 31, 32, n - 1], rng.choice(n, n_sample, replace=False)]))
        tix = torch.as_tensor(idx, device="cuda")
        orcs = {int(i): OracleEnv(spec) for i in idx}
        for i in idx:
            orcs[int(i)].reset(seed + int(i))
        tails = {int(i): env.env_state(int(i))["car_tail"] for i in idx}
        for t in range(steps):
            acts = np.where(rng.random(n) < 0.93, 4, rng.integers(0, 9, n)).astype(np.uint8)
            env.step(torch.as_tensor(acts, device="cuda"))
            torch.cuda.synchronize()
            m = env.obs_map.index_select(0, tix).cpu().numpy()
            rew = env.reward.index_select(0, tix).cpu().numpy()
            term = env.terminated.index_select(0, tix).cpu().numpy()
            for j, i in enumerate(idx):
                i = int(i)
                o = orcs[i]
                r = o.step(int(acts[i]))
                tag = f"t{t} env{i}"
                if rew[j] != r["reward"] or bool(term[j]) != r["terminated"]:
                    bad.append(tag + " reward/terminated")
                reset = r["terminated"]
                if reset:
                    r = o.reset(None)
                if not np.array_equal(m[j], r["obs"]):
                    bad.append(tag + " obs")
                st = env.env_state(i)
                if not reset and st["car_tail"] < tails[i]:
                    compactions += 1
                tails[i] = st["car_tail"]
                max_tail = max(max_tail, st["car_tail"])
                if t % 3 == 2 or t == steps - 1:
                    oc = o.cars()
                    max_cars = max(max_cars, len(oc))
                    if not np.array_equal(env.cars(i), oc):
                        bad.append(tag + " cars")
            if len(bad) > 20:
                break
    finally:
        env.close()
    return bad, compactions, max_tail, max_cars


@pytest.mark.timeout(600)
def test_compaction_keeps_list_order():
    bad, comp, max_tail, max_cars = cautious_rollout(3, 3, 0.5, 2048, 150, 40, 31)
    assert not bad, bad[:10]
    assert comp > 0 and max_cars > 40, (comp, max_tail, max_cars)


@pytest.mark.timeout(600)
def test_compaction_5x5_bench_density():
    bad, comp, max_tail, max_cars = cautious_rollout(5, 5, 0.5, 4096, 120, 24, 5)
    assert not bad, bad[:10]
    assert comp > 0 and max_cars > 200, (comp, max_tail, max_cars)


SCRIPT = r"""
import sys
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
from test_gpu_car_slots import cautious_rollout
bad, comp, max_tail, max_cars = cautious_rollout(3, 3, 0.5, 1024, 120, 32, 8)
print("BAD", len(bad), bad[:5], "compactions", comp, "max_tail", max_tail, "max_cars", max_cars)
sys.exit(1 if bad or comp == 0 else 0)
"""


@pytest.mark.timeout(600)
def test_compaction_with_saturating_counters():
    from pgtg_amd.build import build, variant_path
    build(variant="occsat")
    env = dict(os.environ, PGTG_LIB=variant_path("occsat"))
    code = SCRIPT.format(root=ROOT, tests=os.path.join(ROOT, "tests"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=560)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
