"""Multi-GPU sharding of the batched environment (one process per GPU, torch.distributed).

The path shards embarrassingly: env g of the global batch lives on rank g // n_local and is seeded
with seed_base + g, so an N-GPU run reproduces the single-GPU trajectories of the same global
envs exactly.  The only collectives are all-reduces of a few counters (RCCL over xGMI with the
"nccl" backend on MI355X; gloo on CPU for tests) -- no data-path exchange exists.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    n_local: int

    @property
    def offset(self) -> int:
        """global index of this rank's env 0 (== its seed offset)"""
        return self.rank * self.n_local

    @property
    def n_global(self) -> int:
        return self.world * self.n_local

    def global_ids(self, local_ids):
        return [self.offset + i for i in local_ids]


def from_env(n_local: int) -> Shard:
    return Shard(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(n_local))


def reduce_counters(env_steps: int, episodes: int, elapsed_s: float, device=None,
                    force: bool = False) -> tuple[int, int, float]:
    """(sum env-steps, sum episodes, max elapsed) over ranks; identity without a process group.
    `force`: run the collectives even in a one-rank group (exercises RCCL init and the device
    all-reduce on a one-GPU box)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or (dist.get_world_size() == 1 and not force):
        return int(env_steps), int(episodes), float(elapsed_s)
    cnt = torch.tensor([env_steps, episodes], dtype=torch.int64, device=device)
    tim = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
    dist.all_reduce(tim, op=dist.ReduceOp.MAX)
    return int(cnt[0].item()), int(cnt[1].item()), float(tim[0].item())


def reduce_sum(values, device=None, force: bool = False) -> list[int]:
    """Element-wise sum of integer counters over ranks (identity without a process group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or (dist.get_world_size() == 1 and not force):
        return [int(v) for v in values]
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]
