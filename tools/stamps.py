"""Diagnostic: per-phase wave cycles of k_env from the -DPGTG_STAMPS build (not the product)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pgtg_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), "libpgtg_hip_stamps.so")
from pgtg_amd.vector import PGTGVecEnv  # noqa: E402

names = ["stage", "step", "final", "reset", "store", "obs"]
for N, kw in [(4096, dict(random_map_width=3, random_map_height=3)),
              (131072, dict(random_map_width=5, random_map_height=5))]:
    env = PGTGVecEnv(N, device=0, **kw)
    env.reset(seed=0)
    for k in range(30):
        env.step_random(1, k)
    torch.cuda.synchronize()
    E = 64 if N <= 65536 else 256
    nw = (N + E - 1) // E * 4
    buf = np.zeros(nw * 16, np.uint64)
    _abi.lib().pgtg_read_stamps.argtypes = [C.c_void_p, C.c_uint64]
    _abi.lib().pgtg_read_stamps(buf.ctypes.data, buf.size)
    st = buf.reshape(nw, 16).astype(np.int64)
    d = np.diff(st[:, :7], axis=1)
    print(N, kw, "mean cycles per phase:", {n: int(x) for n, x in zip(names, d.mean(0))},
          "total", int((st[:, 6] - st[:, 0]).mean()), flush=True)
    f = np.diff(st[:, 8:13], axis=1)
    print("   reset (waves with a reset):", {n: int(x) for n, x in zip(["seed", "generate", "compile", "start"], f.mean(0))}, flush=True)
    g = st[:, [9, 13, 14, 15, 10]]
    print("   generate:", {n: int(x) for n, x in zip(["start/goal", "edge init", "removal loop", "tiles+border+obst"], np.diff(g, axis=1).mean(0))}, flush=True)
    env.close()
