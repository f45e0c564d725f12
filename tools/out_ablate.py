"""Diagnostic: step-kernel time with some outputs detached (pgtg_set_outputs with null pointers),
to price the observation and terminal-observation writes.  Usage: python tools/out_ablate.py [cfg5|cfg4|cfg2]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pgtg_amd.vector import PGTGVecEnv, _check  # noqa: E402

CASES = {"cfg2": (4096, dict(random_map_width=3, random_map_height=3)),
         "cfg5": (131072, dict(random_map_width=5, random_map_height=5)),
         "cfg4": (262144, dict(random_map_width=3, random_map_height=3))}


def timed(env, n=100, k0=0):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for k in range(n):
        env.step_random(1, k0 + k)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for name in sys.argv[1:] or ["cfg5"]:
    N, kw = CASES[name]
    env = PGTGVecEnv(N, device=0, **kw)
    env.reset(seed=0)
    timed(env, 30)
    full = env._outs
    res = {"all": timed(env, 100, 100)}
    for label, drop in [("no_final_obs", ["final_obs"]), ("no_obs", ["obs"]), ("no_obs_no_final", ["obs", "final_obs"])]:
        o = type(full)()
        C.memmove(C.byref(o), C.byref(full), C.sizeof(o))
        for f in drop:
            setattr(o, f, None)
        _check(env._lib.pgtg_set_outputs(env._h, C.byref(o)), env._h)
        res[label] = timed(env, 100, 1000)
        _check(env._lib.pgtg_set_outputs(env._h, C.byref(full)), env._h)
    print(name, {k: round(v, 1) for k, v in res.items()}, "us/step", flush=True)
    env.close()
