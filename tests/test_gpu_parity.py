"""HIP product path vs the reference's golden vectors (bit-exact), through the C ABI."""
import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

NO_TRAFFIC = [n for n in helpers.traj_names() if not helpers.has_traffic(helpers.load_traj(n)["meta"])]


@pytest.mark.parametrize("name", NO_TRAFFIC)
def test_golden_trajectory(name):
    d = helpers.load_traj(name)
    bad = helpers.replay_vec(d)
    assert not bad, bad[:10]
