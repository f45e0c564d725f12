#!/usr/bin/env python3
"""Map-generation latency microbenchmark (stamps build only): k_gen_bench runs generate_map +
compile_path `reps` times per lane of a few waves (one wave per SIMD at the default 1 024 envs), and
records per wave the cycles of each part (s_memtime).  The k_envq helper wave's chain is one such map
per lane, so this is the number to shorten.  Usage: python tools/genbench.py [width] [envs] [reps]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from pgtg_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.environ.get("PGTG_STAMPS_LIB") or os.path.join(os.path.dirname(_abi.LIB_PATH), "libpgtg_hip_stamps.so")
from pgtg_amd.vector import PGTGVecEnv  # noqa: E402


def main():
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    env = PGTGVecEnv(n, device=0, random_map_width=w, random_map_height=w)
    env.reset(seed=0)
    L = _abi.lib()
    L.pgtg_gen_bench.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_float)]
    L.pgtg_read_stamps.argtypes = [C.c_void_p, C.c_uint64]
    ms = C.c_float()
    for active in (64, 64):  # (first launch warms up)
        rc = L.pgtg_gen_bench(env._h, reps, active, C.byref(ms))
        assert rc == 0, rc
    nw = (n + 255) // 256 * 4
    buf = np.zeros(max(nw * 32, 1 << 21), np.uint64)
    L.pgtg_read_stamps(buf.ctypes.data, buf.size)
    st = buf[:nw * 32].reshape(nw, 32).astype(np.int64)
    tg, tc = st[:, 0] / reps, st[:, 1] / reps
    it, bfs = st[:, 27], st[:, 26]
    print(f"{w}x{w} maps, {n} lanes, {reps} maps per lane: {ms.value * 1e3:.1f} us; per map and wave (cycles): "
          f"generate {tg.mean():.0f} (max {tg.max():.0f}), compile_path {tc.mean():.0f}; "
          f"last removal loop: iterations {it.mean():.1f}, connectivity-test cycles {bfs.mean():.0f}", flush=True)
    env.close()


if __name__ == "__main__":
    main()
