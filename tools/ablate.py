"""Phase ablation of the step kernel on the GPU: time observe-only, reset-all and step launches."""
import sys
import os
import json
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pgtg_amd.vector import PGTGVecEnv  # noqa: E402


def timed(fn, n=100):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for k in range(n):
        fn(k)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


res = {}
for N, kw in [(4096, dict(random_map_width=3, random_map_height=3)),
              (262144, dict(random_map_width=3, random_map_height=3)),
              (131072, dict(random_map_width=5, random_map_height=5))]:
    env = PGTGVecEnv(N, device=0, **kw)
    env.reset(seed=0)
    for k in range(20):
        env.step_random(1, k)
    r = {}
    r["observe"] = timed(lambda k: env.observe())
    r["reset_all"] = timed(lambda k: env._lib.pgtg_reset_unseeded(env._h, None))
    r["step"] = timed(lambda k: env.step_random(1, 100 + k))
    res[f"{N}x{kw['random_map_width']}"] = r
    print(N, kw, {k: round(v, 1) for k, v in r.items()}, flush=True)
    env.close()
print(json.dumps(res))
