#!/usr/bin/env python3
"""Per-launch step-kernel time over the first launches after a seeded reset (HIP event pair per launch):
how long the map-queue rings take to reach their steady state.  Usage: python tools/ramp.py [workload]
[launches] [envs]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    from pgtg_amd.config import make_spec
    from pgtg_amd.vector import PGTGVecEnv
    wl = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
    n_launch = int(sys.argv[2]) if len(sys.argv) > 2 else 80
    _, _, n, kw = bench.WORKLOADS[wl]
    if len(sys.argv) > 3:
        n = int(sys.argv[3])
    kw = dict(kw)
    mes = kw.pop("max_episode_steps", None)  # the TimeLimit wrapper: a PGTGVecEnv argument, not a PGTGEnv kwarg
    env = PGTGVecEnv(n, spec=make_spec(**kw), device=0, autoreset=True, max_episode_steps=mes)
    acts = None
    rows = []
    for rep in range(2):
        env.reset(seed=0)
        acts = env.random_actions(n_launch, 0x5EED)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n_launch + 1)]
        e0 = env.counters()[1]
        ev[0].record()
        for t in range(n_launch):
            env.step_actions(acts[t])
            ev[t + 1].record()
        torch.cuda.synchronize()
        us = [1e3 * ev[t].elapsed_time(ev[t + 1]) for t in range(n_launch)]
        rows.append(us)
        e1 = env.counters()[1]
        print(f"rep {rep}: resets per launch {(e1 - e0) / n_launch:.0f}", flush=True)
    us = [min(a, b) for a, b in zip(*rows)]
    print(json.dumps({"workload": wl, "envs": n, "us_per_launch": [round(x, 1) for x in us]}))
    for a in (0, 5, 10, 25, 50):
        if a < n_launch:
            seg = us[a:min(n_launch, a + 20)]
            print(f"launches {a}-{a + len(seg) - 1}: mean {sum(seg) / len(seg):.1f} us")
    env.close()


if __name__ == "__main__":
    main()
