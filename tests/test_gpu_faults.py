"""Error paths of the kernels: a data-dependent loop whose exit depends on the consistency of the
map masks must end the launch with an error for the env, never spin (the round-4
library's path walk hung on inconsistent 1-wide edge directions).  The test knob tune_fault bit 0
(include/pgtg.h) clears the path walk's north mask on maps whose tile 0 keeps its east exit, so those
paths that need a north move find no direction: those envs report PGTG_E_DEVICE, the others run
normally, and every launch finishes."""
import warnings

import pytest
import torch

import helpers  # noqa: F401
from pgtg_amd import _abi
from pgtg_amd import config as cfg

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(120)
@pytest.mark.parametrize("kw", [dict(random_map_width=5, random_map_height=5),        # k_qfill + k_envq (map queue)
                                dict(random_map_width=3, random_map_height=3, traffic_density=0.3),  # k_env<true> resets
                                dict(random_map_width=12, random_map_height=10)])     # 256-bit masks (BIG)
def test_inconsistent_path_masks_report_device_error(kw):
    from pgtg_amd.vector import PGTGVecEnv
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        spec = cfg.make_spec(**kw)
    N = 4096
    env = PGTGVecEnv(N, spec=spec, device=0, tune={"fault": 1})
    env.reset(seed=0)
    n, code = env.error_count()
    assert 0 < n < N and code == _abi.PGTG_E_DEVICE, (n, code)
    for t in range(5):  # the broken envs keep stepping (and resetting onto broken maps): no launch spins
        env.step_random(3, t)
    torch.cuda.synchronize()  # (what a broken env reports after that is unspecified: its state is not a map's)
    env.close()
    # the same configuration without the knob: no errors
    ok = PGTGVecEnv(N, spec=spec, device=0)
    ok.reset(seed=0)
    for t in range(5):
        ok.step_random(3, t)
    assert ok.error_count() == (0, 0)
    ok.close()
