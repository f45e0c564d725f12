"""Diagnostic: per-workgroup timeline of k_envq (stamps build): env-wave and helper-wave spans,
empty rings and refill demand per workgroup.  Usage: python tools/wg_timeline.py [cfg5|cfg2]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pgtg_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.path.join(os.path.dirname(_abi.LIB_PATH), "libpgtg_hip_stamps.so")
from pgtg_amd.vector import PGTGVecEnv  # noqa: E402

CASES = {"cfg2": (4096, dict(random_map_width=3, random_map_height=3)),
         "cfg5": (131072, dict(random_map_width=5, random_map_height=5))}
name = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
N, kw = CASES[name]
env = PGTGVecEnv(N, device=0, **kw)
E, _ = env.launch_info()
env.reset(seed=0)
for k in range(40):
    env.step_random(1, k)
torch.cuda.synchronize()
nb = (N + E - 1) // E
buf = np.zeros(nb * 4 * 32, np.uint64)
_abi.lib().pgtg_read_stamps.argtypes = [C.c_void_p, C.c_uint64]
_abi.lib().pgtg_read_stamps(buf.ctypes.data, buf.size)
st = buf.reshape(nb, 4, 32).astype(np.int64)
ew = (E + 63) // 64  # env waves; the helper is wave ew
t0 = st[:, :, 0].min()
env_end = st[:, :ew, 6].max(1) - t0
env_start = st[:, :ew, 0].min(1) - t0
hel_end = st[:, ew, 7] - t0
f = st[:, 0, 12]
F0, F1, F2 = f & 0xffff, (f >> 16) & 0xffff, (f >> 32) & 0xffff
span = np.maximum(env_end, hel_end) - env_start
print(f"{name}: {nb} workgroups of {E} envs; kernel span {int(max(env_end.max(), hel_end.max()))} cycles")
print(f"  env waves end: mean {int(env_end.mean())} p90 {int(np.percentile(env_end, 90))} max {int(env_end.max())}")
print(f"  helper end:    mean {int(hel_end.mean())} p90 {int(np.percentile(hel_end, 90))} max {int(hel_end.max())}")
print(f"  workgroups whose helper ends last: {float((hel_end > env_end).mean()):.2f}")
print(f"  empty rings per wg: mean {F0.mean():.2f}, wgs with any {float((F0 > 0).mean()):.2f}; level-1 {F1.mean():.1f} level-2 {F2.mean():.1f}")
late = np.argsort(-np.maximum(env_end, hel_end))[:5]
for b in late:
    print(f"  wg {b}: start {int(env_start[b])} env_end {int(env_end[b])} helper_end {int(hel_end[b])} F {int(F0[b])},{int(F1[b])},{int(F2[b])}")
env.close()
