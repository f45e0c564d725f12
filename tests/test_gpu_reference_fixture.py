"""The reference's own golden fixture replayed on the GPU: COMPLICATED_ENVIRONMENT
(tests/test_data/reproducibility_data.py:5-2317, replayed by the reference in
tests/test_integration.py:66-93), committed as tests/golden/ref_complicated_environment.npz.  The
same comparison as tests/test_oracle_golden.py for the CPU restatement: the fixture predates the
fork's traffic model, so traffic is disabled (car_rng is an independent stream: maps, obstacles and
the agent's trajectory are unaffected) and the traffic channel and the final traffic crash (step
25) are not compared.  Runs through the single-env facade and through a batch whose every env
replays the fixture at a different lane / workgroup position."""
import json
import os

import numpy as np
import pytest
import torch

import helpers

pytestmark = pytest.mark.gpu


def _fixture():
    z = np.load(os.path.join(helpers.GOLDEN, "ref_complicated_environment.npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    kw = dict(meta["kwargs"])
    kw["traffic_density"] = 0
    spec = helpers.spec_for({"kwargs": kw, "map_file": None})
    perm = helpers.channel_perm(spec, meta["keys"])
    keep = [i for i, k in enumerate(meta["keys"]) if k != "traffic"]
    for k in ("random_map_start_position", "random_map_goal_position", "traffic_light_phases_duration"):
        if isinstance(kw.get(k), list):
            kw[k] = tuple(kw[k])
    return z, meta, spec, perm, keep, kw


def test_facade_replays_reference_fixture():
    from pgtg_amd.env import PGTGEnv
    z, meta, spec, perm, keep, kw = _fixture()
    env = PGTGEnv(**kw)
    obs, _ = env.reset(seed=meta["seed"])
    keys = [k for k, _ in spec.channels]

    def stack(o):
        return np.stack([o["map"][k] for k in keys]).astype(np.uint8)

    assert np.array_equal(stack(obs)[perm][keep], z["obs"][0][keep])
    for n, a in enumerate(z["actions"][:24]):
        obs, rew, term, _, _ = env.step(int(a))
        assert np.array_equal(stack(obs)[perm][keep], z["obs"][n + 1][keep]), n
        assert tuple(obs["position"]) == tuple(z["pos"][n + 1]) and tuple(obs["velocity"]) == tuple(z["vel"][n + 1]), n
        assert rew == z["reward"][n] and term == bool(z["terminated"][n]), n
    env.close()


@pytest.mark.parametrize("n", [1, 100, 5000])
def test_batch_replays_reference_fixture(n):
    from pgtg_amd.vector import PGTGVecEnv
    z, meta, spec, perm, keep, _ = _fixture()
    env = PGTGVecEnv(n, spec=spec, device=0, autoreset=False)
    try:
        env.reset(seed=[meta["seed"]] * n)
        m = env.obs_map.cpu().numpy()
        assert all(np.array_equal(m[i][perm][keep], z["obs"][0][keep]) for i in range(n))
        for k, a in enumerate(z["actions"][:24]):
            env.step(torch.full((n,), int(a), dtype=torch.uint8, device="cuda"))
            m = env.obs_map.cpu().numpy()
            pos, vel = env.position.cpu().numpy(), env.velocity.cpu().numpy()
            rew, term = env.reward.cpu().numpy(), env.terminated.cpu().numpy()
            for i in range(n):
                assert np.array_equal(m[i][perm][keep], z["obs"][k + 1][keep]), (k, i)
                assert tuple(pos[i]) == tuple(z["pos"][k + 1]) and tuple(vel[i]) == tuple(z["vel"][k + 1]), (k, i)
                assert rew[i] == z["reward"][k] and bool(term[i]) == bool(z["terminated"][k]), (k, i)
    finally:
        env.close()
