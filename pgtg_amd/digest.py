"""Per-env output digests of a batched rollout, computed on the device.

A digest condenses one env's step outputs into a uint64 (arithmetic mod 2^64, held in int64
tensors): the sum of W(j) over the observation bytes j that are set, W(D + k) times the small
outputs (position, velocity, reward bits, terminated, truncated, next-subgoal direction, cost bits),
for an env that finished this step its terminal observation's set bytes at W(D + 16 + j), and for
traffic handles the car list after the step (`car_term`: every car's id, square, route, profile,
delay and patience in list order, computed on the device by pgtg_car_digest).
W is the splitmix64 finaliser of j + 1.  The CPU restatement computes the same formula
(oracle/pgtg_oracle.c `orc_rollout_digest`), so a whole batch can be compared env by env at every
step without copying observations to the host; sharded runs compare their slices with a
single-GPU run of the same global batch (bench.py --digest).
"""
from __future__ import annotations

_M64 = (1 << 64) - 1


def _w(j: int) -> int:
    z = (j + 1 + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _signed(u: int) -> int:
    return u - (1 << 64) if u >= 1 << 63 else u


CAR_BASE = 1 << 40


def car_term(cars) -> int:
    """Car-list term of an env's digest (uint64 as a Python int): cars = rows (id, x, y, route,
    profile, patience, delay) in list order (PGTGVecEnv.cars / OracleEnv.cars).  The same formula as
    the device kernel k_car_digest and oracle/pgtg_oracle.c dg_cars."""
    d = (len(cars) * _w(CAR_BASE)) & _M64
    for j, (cid, x, y, route, prof, pat, delay) in enumerate(cars):
        pk = (int(cid) & 0xFFFFFFFF) | int(x) << 32 | int(y) << 40 | int(route) << 48 | int(prof) << 53 | int(delay) << 56
        d = (d + (pk + 1) * _w(CAR_BASE + 1 + 2 * j) + (int(pat) & _M64) * _w(CAR_BASE + 2 + 2 * j)) & _M64
    return d


class Digest:
    """Digest of a PGTGVecEnv's current outputs: `step_digest()` -> int64 [N] device tensor."""

    def __init__(self, env, chunk: int = 1 << 15):
        import torch
        self.env = env
        D = env.obs_map[0].numel()
        self.D = D
        dev = env.device
        self.w_obs = torch.tensor([_signed(_w(j)) for j in range(D)], dtype=torch.int64, device=dev)
        self.w_fin = torch.tensor([_signed(_w(D + 16 + j)) for j in range(D)], dtype=torch.int64, device=dev)
        self.w_small = [_signed(_w(D + k)) for k in range(9)]
        self.chunk = chunk

    def _obs_sum(self, obs, w):
        import torch
        n = obs.shape[0]
        flat = obs.reshape(n, -1)
        out = torch.empty(n, dtype=torch.int64, device=obs.device)
        for lo in range(0, n, self.chunk):
            hi = min(n, lo + self.chunk)
            out[lo:hi] = (flat[lo:hi].to(torch.int64) * w).sum(1)
        return out

    def step_digest(self):
        import torch
        e = self.env
        ws = self.w_small
        d = self._obs_sum(e.obs_map, self.w_obs)
        pos, vel = e.position.to(torch.int64), e.velocity.to(torch.int64)
        d += pos[:, 0] * ws[0] + pos[:, 1] * ws[1] + vel[:, 0] * ws[2] + vel[:, 1] * ws[3]
        d += e.reward.view(torch.int64) * ws[4]
        d += e.terminated.to(torch.int64) * ws[5] + e.truncated.to(torch.int64) * ws[6]
        if e.nsd is not None:
            d += e.nsd.to(torch.int64) * ws[7]
        if e.cost is not None:
            d += e.cost.view(torch.int64) * ws[8]
        if e.final_map is not None:
            done = (e.terminated | e.truncated).to(torch.int64)
            d += self._obs_sum(e.final_map, self.w_fin) * done
        if getattr(e, "has_cars", False):
            d += e.car_digest()
        return d
