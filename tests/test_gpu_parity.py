"""HIP product path vs the reference's golden vectors (bit-exact), through the C ABI."""
import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

@pytest.mark.parametrize("name", helpers.traj_names())
def test_golden_trajectory(name):
    d = helpers.load_traj(name)
    bad = helpers.replay_vec(d)
    assert not bad, bad[:10]
