"""Diagnostic: map generation + path compilation cycles per wave in isolation (stamps build).

Usage: python tools/genbench.py [WxH ...]   (default 5x5 3x3)
For each map size: N=131072 envs, 4 reps, `active` lanes per wave in (1, 16, 64); prints the mean
per-wave cycles of generate_map and compile_path per rep and the kernel time."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pgtg_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.environ.get("PGTG_STAMPS_LIB") or os.path.join(os.path.dirname(_abi.LIB_PATH), "libpgtg_hip_stamps.so")
from pgtg_amd.vector import PGTGVecEnv  # noqa: E402

lib = _abi.lib()
lib.pgtg_gen_bench.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_float)]
lib.pgtg_read_stamps.argtypes = [C.c_void_p, C.c_uint64]
N, REPS = 131072, 4
for size in (sys.argv[1:] or ["5x5", "3x3"]):
    w, hgt = (int(t) for t in size.split("x"))
    env = PGTGVecEnv(N, device=0, random_map_width=w, random_map_height=hgt)
    env.reset(seed=0)
    torch.cuda.synchronize()
    for active in (1, 16, 64):
        ms = C.c_float()
        lib.pgtg_gen_bench(env._h, 1, active, C.byref(ms))  # warm
        rc = lib.pgtg_gen_bench(env._h, REPS, active, C.byref(ms))
        assert rc == 0, rc
        nw = N // 64
        buf = np.zeros(nw * 32, np.uint64)
        lib.pgtg_read_stamps(buf.ctypes.data, buf.size)
        st = buf.reshape(nw, 32)
        g, cp = st[:, 0].astype(float) / REPS, st[:, 1].astype(float) / REPS
        print(f"{size} active {active:2d}: generate {g.mean():8.0f} (max {g.max():8.0f})  compile {cp.mean():7.0f} "
              f"cycles/wave/rep; kernel {ms.value:.3f} ms for {REPS} reps", flush=True)
    env.close()
