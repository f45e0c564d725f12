#!/usr/bin/env python3
"""bench.py -- env-steps/s of the batched PGTG hot path (reset+step) on MI355X.

Contract (see DESIGN.md "Measurement"):
  python bench.py --gpus N --steps K --warmup W           (N>1 under torch.distributed.run)
A "step" is one tick of every env of the rank's batch: the step kernel with same-step in-kernel
auto-reset, reading that tick's actions (synthetic uniform policy, 1 B/env, generated on the device
before the timed region) from HBM.  Inputs and state are resident in HBM for the whole timed region.  Each rank owns a contiguous shard of envs (global
env g is seeded with g, weak scaling: per-GPU envs fixed); the only collectives are an RCCL
all-reduce of the device env-step/episode counters and of the elapsed time (max).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (batched random-action rollout) at 1/2/4/8 MI355X"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md

WORKLOADS = {
    # name: (BASELINE.json configs[] index, description, envs per GPU, PGTGEnv kwargs)
    "cfg2": (1, "4096 vectorised envs, default 3x3 procedural map, random actions, auto-reset",
             4096, dict(random_map_width=3, random_map_height=3)),
    "cfg4": (3, "262144 envs, default 3x3 map, random actions, in-kernel auto-reset (map_generator)",
             262144, dict(random_map_width=3, random_map_height=3)),
    "cfg5": (4, "1048576 envs sharded 8x MI355X (131072 5x5-map envs per GPU), random actions, auto-reset, "
                "RCCL-reduced global step counter",
             131072, dict(random_map_width=5, random_map_height=5)),
    "cfg3": (2, "65536 envs, 5x5 procedural map, traffic density 0.5, random actions, auto-reset",
             65536, dict(random_map_width=5, random_map_height=5, traffic_density=0.5)),
}


def algorithmic_bytes(spec, n_envs: int, resets: float, cars_per_env: float = 0.0) -> float:
    """Bytes one step launch must move (DESIGN.md "Algorithmic bytes"): per env-step the action,
    the 32-B agent record read+written, the 2-B/tile plan read, the observation and small outputs
    written; per reset the seed read, the new plan written and the terminal observation written."""
    nt = spec.map_tiles[0] * spec.map_tiles[1]
    obs = len(spec.channels) * spec.window ** 2
    small = 8 + 8 + 8 + 3 + (4 if spec.next_subgoal else 0) + (8 if spec.separate_reward_cost else 0)
    per_step = 1 + 2 * 32 + 2 * nt + obs + small
    per_reset = 8 + 2 * nt + obs + 16 + (4 if spec.next_subgoal else 0)
    if cars_per_env:
        # cars: 12 B per car read + written per step, car_rng state 80 B r/w, traffic record 16 B r/w;
        # resets write the new cars (12 B each) and the spawner list (2 B per spawner, ~nt)
        per_step += 2 * 12 * cars_per_env + 2 * 40 + 2 * 16
        per_reset += 12 * cars_per_env + 2 * nt + 80
    return n_envs * per_step + resets * per_reset


def cpu_baseline(spec, seconds: float = 12.0) -> dict:
    """The CPU oracle (a scalar C port of the reference path; the Python reference itself cannot
    travel to the GPU box) timed on one host core over a bounded sample of the same workload."""
    from oracle import oracle
    oracle.build()
    n_envs, steps = 64, 50
    t0 = time.perf_counter()
    done = oracle.bench(spec, n_envs, steps)
    dt = time.perf_counter() - t0
    reps = max(1, int(seconds / max(dt, 1e-3)))
    t0 = time.perf_counter()
    done = oracle.bench(spec, n_envs * reps, steps)
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"{n_envs * reps} envs x {steps} random-action steps with auto-reset "
                      f"({done} env-steps, {dt:.1f} s) on the C restatement oracle/pgtg_oracle.c"}


def load_traffic(workload: str, launch_bytes_alg: float):
    """HBM bytes per step launch from the committed rocprofv3 PMC summary, if one exists."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=50)
    # Default: BASELINE.json's metric is quoted "at 1/2/4/8 MI355X", i.e. on configs[4] (1 048 576
    # envs of 5x5 maps sharded over 8 GPUs); each rank runs its 131 072-env shard, so N=8 is exactly
    # configs[4] and N=1,2,4 are its weak-scaling prefixes.  cfg2 = configs[1] (4 096 envs, one GPU).
    ap.add_argument("--workload", default="cfg5", choices=sorted(WORKLOADS))
    ap.add_argument("--envs", type=int, default=0, help="override envs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--timing-every", type=int, default=16,
                    help="bracket every n-th step launch with HIP events (kernel duration for the roofline)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for a one-GPU box (never set by the driver): every rank on GPU 0, gloo counters
    backend = os.environ.get("PGTG_BENCH_BACKEND", "nccl")  # nccl == RCCL over xGMI on MI355X
    if os.environ.get("PGTG_BENCH_SAME_GPU") == "1":
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    red_dev = dev if backend == "nccl" else None

    from pgtg_amd.build import build
    build()  # no-op when the in-tree library is current (file-locked across ranks)
    from pgtg_amd.config import make_spec
    from pgtg_amd.dist import Shard, reduce_counters
    from pgtg_amd.vector import PGTGVecEnv

    cfg_idx, desc, n_local, kwargs = WORKLOADS[args.workload]
    if args.envs:
        n_local = args.envs
    spec = make_spec(**kwargs)
    shard = Shard(rank, world, n_local)
    env = PGTGVecEnv(n_local, spec=spec, device=local, autoreset=True)
    env.reset(seed=shard.offset)  # global env g = rank*n_local + i gets seed g
    act_seed = 0x5EED
    # synthetic policy: uniform actions from a counter hash of (seed, env, t), generated before the
    # timed region so that the timed steps read their inputs from HBM like a resident rollout buffer
    actions = env.random_actions(args.warmup + args.steps, act_seed)
    for t in range(args.warmup):
        env.step_actions(actions[t])
    torch.cuda.synchronize(dev)
    steps0, eps0 = env.counters()
    env.enable_timing(args.timing_every)
    env.timing_read(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for t in range(args.warmup, args.warmup + args.steps):
        env.step_actions(actions[t])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms, launches = env.timing_read(reset=True)
    steps1, eps1 = env.counters()
    # RCCL (nccl backend) all-reduce: global env-step / episode counters (sum), slowest rank's time (max)
    total_steps, total_eps, t_max = reduce_counters(steps1 - steps0, eps1 - eps0, elapsed, device=red_dev)
    value = total_steps / t_max

    if rank == 0:
        resets_per_launch = (eps1 - eps0) / max(1, args.steps)
        avg_kernel_s = (kern_ms / max(1, launches)) / 1e3
        cars = env.mean_cars() if spec.traffic_density > 0 else 0.0
        alg = algorithmic_bytes(spec, n_local, resets_per_launch, cars)
        achieved = alg / avg_kernel_s / 1e9 if avg_kernel_s > 0 else 0.0
        rec = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * t_max / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (device uniform random actions, seeds = global env index)",
            "config": {"workload": f"configs[{cfg_idx}]: {desc}", "envs_per_gpu": n_local,
                       "envs_total": n_local * world, "map": f"{spec.width}x{spec.height}",
                       "traffic_density": spec.traffic_density, "autoreset": True,
                       "parallelism": f"dp{world} (env shards, no data-path collective)"},
            "episodes": total_eps,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": load_traffic(args.workload, alg),
                         "kernel": env.step_kernel() + " (step + in-kernel auto-reset)", "avg_kernel_us": avg_kernel_s * 1e6,
                         "alg_bytes_per_launch": alg, "resets_per_launch": resets_per_launch,
                         "envs_per_workgroup": env.launch_info()[0], "lds_bytes": env.launch_info()[1],
                         "workgroups_per_cu": env.occupancy()},
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(spec, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
