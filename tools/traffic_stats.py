"""Diagnostic: distribution of per-env car and spawner counts for a traffic workload on the GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from pgtg_amd.vector import PGTGVecEnv  # noqa: E402

w = int(sys.argv[1]) if len(sys.argv) > 1 else 5
d = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
env = PGTGVecEnv(4096, device=0, random_map_width=w, random_map_height=w, traffic_density=d)
env.reset(seed=0)
for k in range(20):
    env.step_random(3, k)
idx = range(0, 4096, 4)
sp = np.array([env.env_state(i)["n_spawners"] for i in idx])
cars = np.array([env.env_state(i)["n_cars"] for i in idx])
print(f"{w}x{w} density {d}: spawners mean {sp.mean():.1f} p99 {np.percentile(sp, 99):.0f} max {sp.max()}; "
      f"cars mean {cars.mean():.1f} max {cars.max()}")
