"""The CPU oracle is pinned against the reference: its own golden trajectory and the generated
vectors (tests/golden, made by tools/gen_golden.py from the imported reference)."""
import json
import os

import numpy as np
import pytest

import helpers
from oracle.oracle import OracleEnv


@pytest.mark.parametrize("name", helpers.traj_names())
def test_oracle_matches_reference_trajectory(name):
    d = helpers.load_traj(name)
    bad = helpers.replay_oracle(d)
    assert not bad, bad[:10]


def test_oracle_matches_reference_reproducibility_fixture():
    """tests/test_data/reproducibility_data.py (COMPLICATED_ENVIRONMENT, 25 steps).  The fixture
    predates the fork's traffic model, so traffic is disabled here (car_rng is an independent
    stream, so maps, obstacles and the agent trajectory are unaffected) and the traffic channel and
    the final traffic crash (step 25) are not compared."""
    z = np.load(os.path.join(helpers.GOLDEN, "ref_complicated_environment.npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    kw = dict(meta["kwargs"])
    kw["traffic_density"] = 0
    spec = helpers.spec_for({"kwargs": kw, "map_file": None})
    perm = helpers.channel_perm(spec, meta["keys"])
    keep = [i for i, k in enumerate(meta["keys"]) if k != "traffic"]
    env = OracleEnv(spec)
    r = env.reset(meta["seed"])
    assert np.array_equal(r["obs"][perm][keep], z["obs"][0][keep])
    for n, a in enumerate(z["actions"][:24]):
        r = env.step(int(a))
        assert np.array_equal(r["obs"][perm][keep], z["obs"][n + 1][keep]), n
        assert tuple(r["pos"]) == tuple(z["pos"][n + 1]) and tuple(r["vel"]) == tuple(z["vel"][n + 1])
        assert r["reward"] == z["reward"][n] and r["terminated"] == bool(z["terminated"][n])
