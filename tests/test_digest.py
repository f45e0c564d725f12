"""The device digest formula (pgtg_amd/digest.py, torch) equals the restatement's
(oracle/pgtg_oracle.c orc_rollout_digest, C) on the same outputs, so the exhaustive GPU parity tests
can compare whole batches digest by digest.  Runs on CPU tensors (no GPU needed)."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import helpers  # noqa: F401
from oracle import oracle
from oracle.oracle import OracleEnv
from pgtg_amd import config as cfg
from pgtg_amd.digest import Digest, car_term

M64 = (1 << 64) - 1


def action(seed: int, t: int, g: int) -> int:
    z = seed ^ ((t * 0x9E3779B97F4A7C15) & M64) ^ ((g * 0xD1B54A32D192ED03) & M64)
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    return ((z >> 32) * 9) >> 32


@pytest.mark.parametrize("kw", [
    dict(random_map_width=3, random_map_height=3),
    dict(random_map_width=4, random_map_height=4, use_next_subgoal_direction=True, separate_reward_cost=True,
         random_map_obstacle_probability=0.5, standing_still_penalty=0.5),
    dict(random_map_width=3, random_map_height=3, traffic_density=0.3, use_sliding_observation_window=True),
    dict(random_map_width=4, random_map_height=3, traffic_density=0.5),
])
def test_digest_formula_matches_oracle(kw):
    spec = cfg.make_spec(**kw)
    N, T, off, seed = 24, 30, 1000, 0xA11CE
    ref = oracle.rollout_digest(spec, N, T, seed, env_offset=off, threads=2)
    envs = [OracleEnv(spec) for _ in range(N)]
    first = [e.reset(off + i) for i, e in enumerate(envs)]
    D = first[0]["obs"].size
    fake = SimpleNamespace(device=torch.device("cpu"), obs_map=torch.zeros((N,) + first[0]["obs"].shape, dtype=torch.uint8))
    dg = Digest(fake)
    assert dg.D == D
    for t in range(T):
        rs, fin = [], np.zeros((N,) + first[0]["obs"].shape, np.uint8)
        for i, e in enumerate(envs):
            r = e.step(action(seed, t, off + i))
            if r["terminated"]:
                fin[i] = r["obs"]
                nr = e.reset(None)
                r = dict(nr, reward=r["reward"], cost=r["cost"], terminated=True, truncated=r["truncated"])
            rs.append(r)
        fake.obs_map = torch.as_tensor(np.stack([r["obs"] for r in rs]))
        fake.final_map = torch.as_tensor(fin)
        fake.position = torch.tensor([r["pos"] for r in rs], dtype=torch.int32)
        fake.velocity = torch.tensor([r["vel"] for r in rs], dtype=torch.int32)
        fake.reward = torch.tensor([r["reward"] for r in rs], dtype=torch.float64)
        fake.terminated = torch.tensor([r["terminated"] for r in rs])
        fake.truncated = torch.tensor([r["truncated"] for r in rs])
        fake.nsd = torch.tensor([r["nsd"] for r in rs], dtype=torch.int32) if spec.next_subgoal else None
        fake.cost = torch.tensor([r["cost"] for r in rs], dtype=torch.float64) if spec.separate_reward_cost else None
        fake.has_cars = spec.traffic_density > 0
        terms = [car_term(e.cars()) for e in envs]
        fake.car_digest = lambda: torch.tensor(np.array(terms, dtype=np.uint64).view(np.int64))
        got = dg.step_digest().numpy().view(np.uint64)
        assert np.array_equal(got, ref[t]), f"t{t}: {np.nonzero(got != ref[t])[0][:5]}"
