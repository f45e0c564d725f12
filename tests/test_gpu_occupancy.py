"""4-bit occupancy counters with exact recount: the traffic trajectories replayed through a build
whose counters saturate at 2 cars (pgtg_amd/build.py VARIANTS["occsat"]), so that the recount path
runs on nearly every step, must stay bit-exact.  Runs in a subprocess (one library per process)."""
import os
import subprocess
import sys

import pytest

import helpers

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
import helpers
bad = []
for name in {names!r}:
    bad += [name + ": " + b for b in helpers.replay_vec(helpers.load_traj(name))]
print("BAD", len(bad), bad[:5])
sys.exit(1 if bad else 0)
"""


def test_saturating_counters_stay_exact():
    from pgtg_amd.build import build, variant_path
    build(variant="occsat")
    names = [n for n in helpers.traj_names() if helpers.has_traffic(helpers.load_traj(n)["meta"])]
    assert names
    env = dict(os.environ, PGTG_LIB=variant_path("occsat"))
    code = SCRIPT.format(root=ROOT, tests=os.path.join(ROOT, "tests"), names=names)
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
