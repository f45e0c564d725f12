"""Multi-rank sharding and counter reduction (gloo, world_size 2, CPU).  On MI355X the same code
runs with the nccl (= RCCL) backend, one process per GPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pgtg_amd.dist import Shard, reduce_counters, reduce_sum


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_local, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = Shard(rank, world, n_local)
    steps, eps = n_local * 10, rank + 3
    tot_steps, tot_eps, t = reduce_counters(steps, eps, 1.0 + rank)
    maps = reduce_sum([100 * (rank + 1), rank])
    q.put((rank, sh.offset, sh.global_ids([0, n_local - 1]), tot_steps, tot_eps, t, maps))
    dist.destroy_process_group()


def test_two_rank_shards_and_counters():
    world, n_local = 2, 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_local, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [0, n_local]
    assert res[1][2] == [n_local, 2 * n_local - 1]  # contiguous global ids == seeds
    for r in res:
        assert r[3] == world * n_local * 10 and r[4] == 3 + 4 and r[5] == 2.0
        assert r[6] == [300, 1]


def test_single_process_identity():
    assert reduce_counters(5, 2, 0.5) == (5, 2, 0.5)
    assert reduce_sum([7, 9]) == [7, 9]
