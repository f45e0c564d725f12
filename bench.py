#!/usr/bin/env python3
"""bench.py -- env-steps/s of the batched PGTG hot path (reset+step) on MI355X.

Contract (see DESIGN.md "Measurement"):
  python bench.py --gpus N --steps K --warmup W           (N>1 under torch.distributed.run)
A "step" is one tick of every env of the batch: the step kernel with same-step in-kernel auto-reset,
reading that tick's actions (synthetic uniform policy, 1 B/env, generated on the device before the
timed region) from HBM.  Inputs and state are resident in HBM for the whole timed region.

The default workload is BASELINE.json configs[4], the config its metric is quoted on: 1 048 576
envs of 5x5 maps.  The batch is fixed and split over the ranks (strong scaling): rank r owns the
contiguous shard of envs_total / N envs starting at global env r * envs_total / N, seeded with the
global index and driven by the actions of the global index, so every N runs the same 1 048 576
trajectories (bench.py --digest checks that a sharded run's outputs equal a single-GPU run's).  The
only collectives are an RCCL all-reduce of the device env-step/episode counters and of the elapsed
time (max).  Prints ONE JSON line on rank 0.
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
PEAK_HBM_SPEC_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
PEAK_HBM_GUIDE_GBS = 6290.0  # the same guide's measured float4 copy (79 % of spec)

WORKLOADS = {
    # name: (BASELINE.json configs[] index, description, envs of the whole batch, PGTGEnv kwargs)
    "cfg2": (1, "4096 vectorised envs, default 3x3 procedural map, random actions, auto-reset",
             4096, dict(random_map_width=3, random_map_height=3)),
    "cfg4": (3, "262144 envs, default 3x3 map, random actions, in-kernel auto-reset (map_generator)",
             262144, dict(random_map_width=3, random_map_height=3)),
    "cfg5": (4, "1048576 envs of 5x5 procedural maps split over the GPUs, random actions, auto-reset, "
                "RCCL-reduced global step counter",
             1048576, dict(random_map_width=5, random_map_height=5)),
    "cfg3": (2, "65536 envs, 5x5 procedural map, traffic density 0.5, random actions, auto-reset",
             65536, dict(random_map_width=5, random_map_height=5, traffic_density=0.5)),
    # not a BASELINE config: the reference's own caller (pgtg/train.py:21-40, PGTGEnv kwargs + TimeLimit(100))
    # at a GPU-sized batch -- the generic observation path (sliding window, next-subgoal direction),
    # obstacles and traffic together
    "train": (None, "65536 envs with pgtg/train.py's PGTGEnv settings: 4x4 maps, obstacles 0.2, connections 0.8, "
                    "traffic 0.2, driver mix 15/50/20/10/5, sliding window 5, next-subgoal direction, TimeLimit(100)",
              65536, dict(random_map_width=4, random_map_height=4, random_map_obstacle_probability=0.2,
                          random_map_percentage_of_connections=0.8, traffic_density=0.2,
                          conservative_driver_percentage=0.15, normal_driver_percentage=0.50,
                          aggressive_driver_percentage=0.20, elderly_driver_percentage=0.10,
                          reckless_driver_percentage=0.05, sliding_observation_window_size=5,
                          max_allowed_deviation=15, use_sliding_observation_window=True,
                          use_next_subgoal_direction=True, final_goal_bonus=200, standing_still_penalty=1,
                          max_episode_steps=100)),
}


def algorithmic_bytes(spec, n_envs: int, resets: float, cars_per_env: float = 0.0) -> float:
    """Bytes one step launch must move, SURVEY.md section 8(d)'s model:
    per env-step B = 1 (action) + 2*18 (agent state r+w) + 2*H*W (tile plan r) + obs (channels x
    window^2 int8 + 2 x 2 int32) + 10 (reward f64 + 2 flags) [+ 2*80 car_rng r+w + 2*10*C cars r+w];
    per reset 2*H*W (plan) + 5*40 (RNG streams) + 18 (agent) + 10*C (cars) + obs (terminal obs)."""
    nt = spec.map_tiles[0] * spec.map_tiles[1]
    obs = len(spec.channels) * spec.window ** 2 + 16
    per_step = 1 + 2 * 18 + 2 * nt + obs + 10
    per_reset = 2 * nt + 5 * 40 + 18 + obs
    if cars_per_env:
        per_step += 2 * 80 + 2 * 10 * cars_per_env
        per_reset += 10 * cars_per_env
    return n_envs * per_step + resets * per_reset


def cpu_baseline(spec, seconds: float = 15.0) -> dict:
    """The CPU restatement (oracle/pgtg_oracle.c, a scalar C port of the reference path; the Python
    reference itself cannot travel to the GPU box) timed on the host cores this process may use,
    one thread per core over disjoint env ranges, on a bounded sample of the same workload."""
    from oracle import oracle
    oracle.build()
    threads = oracle.host_threads()
    n_envs, steps = 32 * threads, 50
    t0 = time.perf_counter()
    oracle.bench_parallel(spec, n_envs, steps, threads)
    dt = time.perf_counter() - t0
    reps = max(1, int(seconds / max(dt, 1e-3)))
    t0 = time.perf_counter()
    done = oracle.bench_parallel(spec, n_envs * reps, steps, threads)
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "label": "restatement",
            "sample": f"{n_envs * reps} envs x {steps} random-action steps with auto-reset "
                      f"({done} env-steps, {dt:.1f} s) on the C restatement oracle/pgtg_oracle.c, "
                      f"{threads} host threads"}


def measure_hbm(device: int) -> float:
    """Measured HBM denominator: a 16-B/lane stream copy between two 2 GiB buffers (pgtg_measure_hbm),
    (read + write) GB/s."""
    import ctypes as C

    from pgtg_amd import _abi
    gbs = C.c_double()
    rc = _abi.lib().pgtg_measure_hbm(device, 2 << 30, 20, C.byref(gbs))
    return gbs.value if rc == 0 else 0.0


def load_traffic(workload: str, n_envs: int):
    """HBM bytes per step launch from the committed rocprofv3 PMC summary of this workload at this
    batch size (profiles/pmc_<workload>.json, tools/pmc.py), and the file it came from."""
    p = os.path.join("profiles", f"pmc_{workload}.json")
    try:
        with open(os.path.join(ROOT, p)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if d.get("envs") not in (None, n_envs):
        return None, None
    return d.get("hbm_bytes_per_launch"), p


# Issue roofline: one instruction per SIMD per cycle at the 2 400 MHz engine clock (MI355X_MICROARCH.md:
# 256 CUs x 4 SIMDs), and the VALU's own ceiling (a wave64 VALU instruction issues over 2 cycles)
PEAK_ISSUE = 256 * 4 * 2.4e9
PEAK_VALU = PEAK_ISSUE / 2


def load_issue(workload: str, n_envs: int, avg_kernel_s: float):
    """Issue roofline from the committed SQ counters of this workload (profiles/sq_<workload>.json,
    tools/sq_json.py): executed VALU + SALU wave-instructions of the step's kernels per launch over the
    average launch duration measured in this run."""
    p = os.path.join("profiles", f"sq_{workload}.json")
    try:
        with open(os.path.join(ROOT, p)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("envs") != n_envs or avg_kernel_s <= 0:
        return None
    valu = sum(k.get("SQ_INSTS_VALU", 0.0) for k in d["kernels"].values())
    salu = sum(k.get("SQ_INSTS_SALU", 0.0) for k in d["kernels"].values())
    insts = valu + salu
    return {"bound": "issue", "unit": "wave-instructions/s", "achieved": insts / avg_kernel_s, "peak": PEAK_ISSUE,
            "frac": insts / avg_kernel_s / PEAK_ISSUE, "valu_frac": valu / avg_kernel_s / PEAK_VALU,
            "valu_per_launch": valu, "salu_per_launch": salu, "insts_per_env_step": insts / n_envs,
            "peak_model": "256 CU x 4 SIMD x 2.4 GHz, one instruction per SIMD-cycle (VALU: one per 2)",
            "kernels": sorted(d["kernels"]), "source": p}


# the stamps count shader cycles (s_memtime) at the
# engine clock, 2.4 GHz (MI355X_MICROARCH.md)
ENGINE_GHZ = 2.4


def load_latency(workload: str, n_envs: int, avg_kernel_s: float):
    """Latency bound for the launches whose workgroups are a single round of long serial chains (the
    configs[1] batch: 16 envs per workgroup, one workgroup per CU): the measured per-wave chain of the
    step kernel (profiles/stamps_<workload>.json, tools/stamps.py on the -DPGTG_STAMPS build) at the
    engine clock against the measured launch duration.  frac = chain time / launch time: 1.0 means the
    launch is exactly one wave's chain long, so only a shorter chain makes it faster."""
    p = os.path.join("profiles", f"stamps_{workload}.json")
    try:
        with open(os.path.join(ROOT, p)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("envs") != n_envs or avg_kernel_s <= 0:
        return None
    chain_us = d["wave_chain_cycles_mean"] / (ENGINE_GHZ * 1e3)
    chain_max_us = d["wave_chain_cycles_max"] / (ENGINE_GHZ * 1e3)
    return {"bound": "latency", "unit": "us", "chain_cycles_mean": d["wave_chain_cycles_mean"],
            "chain_cycles_max": d["wave_chain_cycles_max"], "engine_ghz": ENGINE_GHZ, "chain_us_mean": chain_us,
            "chain_us_max": chain_max_us, "avg_kernel_us": avg_kernel_s * 1e6,
            "frac": chain_us / (avg_kernel_s * 1e6), "frac_max": chain_max_us / (avg_kernel_s * 1e6),
            "phases_mean_cycles": d.get("phases_mean_cycles"), "source": p}


def adapter_bench(args) -> None:
    """The reference caller's interface (pgtg/train.py:39-55: TimeLimit(100) -> FlattenObservation ->
    SubprocVecEnv) served by PGTGSB3VecEnv: K steps of step_async/step_wait with the flattened
    observation vectors, rewards, dones and infos returned -- as host numpy arrays (SB3's VecEnv
    contract) or as device tensors (`device_obs=True`).  Actions: uniform random, pre-generated (host
    array or device tensor).  Not a BASELINE metric; one JSON line."""
    import numpy as np
    import torch

    from pgtg_amd.build import build
    build()
    from pgtg_amd.sb3 import PGTGSB3VecEnv
    _, desc, n, kwargs = WORKLOADS["train"]
    n = args.envs or n
    kwargs = dict(kwargs)
    mes = kwargs.pop("max_episode_steps", 100)
    dev = args.adapter == "device"
    env = PGTGSB3VecEnv(n, max_episode_steps=mes, device=0, seed=0, device_obs=dev, **kwargs)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(12345)
    acts = torch.randint(0, 9, (args.warmup + args.steps, n), device="cuda", dtype=torch.uint8, generator=g)
    host_acts = None if dev else acts.cpu().numpy()
    a = (lambda t: acts[t]) if dev else (lambda t: host_acts[t])
    for t in range(args.warmup):
        env.step(a(t))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = 0
    monitor = args.adapter == "host-monitor"
    ep_ret, ep_len = np.zeros(n), np.zeros(n, np.int64)
    for t in range(args.warmup, args.warmup + args.steps):
        obs, rew, dones, infos = env.step(a(t))
        if monitor:  # stable_baselines3 VecMonitor.step_wait: returns, lengths, list(infos[:]), episode dicts
            ep_ret += rew
            ep_len += 1
            new_infos = list(infos[:])
            for i in np.nonzero(dones)[0]:
                info = dict(infos[i])
                info["episode"] = {"r": ep_ret[i], "l": ep_len[i], "t": 0.0}
                new_infos[i] = info
                ep_ret[i] = 0
                ep_len[i] = 0
                done += 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rec = {"metric": "env-steps/sec through the SB3 VecEnv adapter (PGTGSB3VecEnv.step_async/step_wait)",
           "value": n * args.steps / dt, "unit": "env-steps/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True,
           "path": ("device tensors (device_obs=True): flattened obs, rewards, dones and terminal "
                    "observations stay in HBM" if dev else
                    "host numpy (SB3's VecEnv contract): flattened float32 obs copied to the host every step"
                    + (", plus VecMonitor's per-step host work (list(infos[:]), episode dicts)" if monitor else "")),
           "obs_dim": env.obs_dim, "obs_bytes_per_step": n * env.obs_dim * 4,
           "data": "synthetic (uniform random actions, seeds 0..N-1)",
           "config": {"workload": "caller: " + desc, "envs": n, "adapter": args.adapter}}
    print(json.dumps(rec), flush=True)
    env.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)  # T >= 1000 after a 50-step warm-up
    ap.add_argument("--warmup", type=int, default=50)
    # Default: configs[4] (1 048 576 envs of 5x5 maps), the config BASELINE.json's metric is quoted
    # on, split over the N GPUs.  cfg2/cfg4/cfg3 = configs[1]/[3]/[2] (single-GPU configs).
    ap.add_argument("--workload", default="cfg5", choices=sorted(WORKLOADS))
    ap.add_argument("--envs", type=int, default=0, help="override the batch (envs over all GPUs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group and run the counter all-reduce on the device even "
                         "at world size 1 (RCCL check on a one-GPU box; use under torch.distributed.run)")
    ap.add_argument("--digest", default="",
                    help="after the timed window, run --digest-steps more steps and save each rank's per-env "
                         "output digests to <path>.rank<r>.npz (tools/digest_compare.py)")
    ap.add_argument("--digest-steps", type=int, default=8)
    ap.add_argument("--per-step", action="store_true", help="A/B: one pgtg_step host call per timed step")
    ap.add_argument("--envs-per-block", type=int, default=0, help="A/B: force the step kernel's envs per workgroup")
    ap.add_argument("--kt-wpc", type=int, default=0, help="A/B: k_traffic workgroups per CU")
    ap.add_argument("--kt-cap", type=int, default=0, help="A/B: k_traffic envs per wave held in LDS")
    ap.add_argument("--queue-mode", type=int, default=0,
                    help="A/B: map-queue step kernel (0 automatic, 1 k_envq persistent, 2 k_envb per block)")
    ap.add_argument("--adapter", choices=["host", "host-monitor", "device"], default="",
                    help="time the SB3 VecEnv adapter (pgtg_amd/sb3.py) instead: PGTGSB3VecEnv.step over "
                         "the caller workload (pgtg/train.py's settings), host numpy or device-tensor path; "
                         "host-monitor adds SB3 VecMonitor's per-step host work (pgtg/train.py:55)")
    args = ap.parse_args()
    if args.adapter:
        return adapter_bench(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for a one-GPU box (never set by the driver): every rank on GPU 0, gloo counters
    backend = os.environ.get("PGTG_BENCH_BACKEND", "nccl")  # nccl == RCCL over xGMI on MI355X
    if os.environ.get("PGTG_BENCH_SAME_GPU") == "1":
        local = 0
    use_dist = world > 1 or args.dist
    if use_dist:
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    red_dev = dev if backend == "nccl" else None

    from pgtg_amd.build import build
    build()  # no-op when the in-tree library is current (file-locked across ranks)
    from pgtg_amd.config import make_spec
    from pgtg_amd.dist import Shard, reduce_counters, reduce_sum
    from pgtg_amd.vector import PGTGVecEnv

    cfg_idx, desc, n_total, kwargs = WORKLOADS[args.workload]
    if args.envs:
        n_total = args.envs
    if n_total % world:
        raise SystemExit(f"{n_total} envs do not split evenly over {world} ranks")
    n_local = n_total // world
    kwargs = dict(kwargs)
    max_steps = kwargs.pop("max_episode_steps", None)
    spec = make_spec(**kwargs)
    shard = Shard(rank, world, n_local)
    peak_copy = measure_hbm(local) if rank == 0 else 0.0
    tune = {k: v for k, v in (("envs_per_block", args.envs_per_block), ("kt_wpc", args.kt_wpc),
                              ("kt_cap", args.kt_cap), ("queue_mode", args.queue_mode)) if v} or None
    env = PGTGVecEnv(n_local, spec=spec, device=local, autoreset=True, max_episode_steps=max_steps, tune=tune)
    env.reset(seed=shard.offset)  # global env g = rank*n_local + i gets seed g
    act_seed = 0x5EED
    # synthetic policy: uniform actions from a counter hash of (seed, global env, t), generated before
    # the timed region so that the timed steps read their inputs from HBM like a resident rollout buffer
    actions = env.random_actions(args.warmup + args.steps, act_seed, env_offset=shard.offset)
    for t in range(args.warmup):
        env.step_actions(actions[t])
    torch.cuda.synchronize(dev)
    steps0, eps0 = env.counters()
    maps0 = env.queue_maps()
    env.enable_timing(0)  # no per-launch events inside the timed window
    # one event pair around the whole window on the stream the kernels run on (torch's current
    # stream, which the env binds): the device time of the K launches, launch gaps included
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record()
    if args.per_step:
        for t in range(args.warmup, args.warmup + args.steps):
            env.step_actions(actions[t])
    else:  # one host call queues the K launches (pgtg_step_many), same kernels and results
        env.step_many(actions[args.warmup:args.warmup + args.steps])
    ev1.record()
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    window_ms = ev0.elapsed_time(ev1)
    steps1, eps1 = env.counters()
    maps1 = env.queue_maps()
    # the step kernel's average launch duration for the roofline: the event pair around the timed
    # window divided by the launches (back-to-back launches on one stream: the window is their device
    # time; it agrees with rocprofv3's per-kernel average to < 0.5 %, profiles/r04/f2, while brackets
    # around single launches add their own gaps: +24 % on the 22-us configs[1] kernel)
    kern_ms, launches = window_ms, args.steps
    # RCCL (nccl backend) all-reduce: global env-step / episode counters (sum), slowest rank's time (max)
    total_steps, total_eps, t_max = reduce_counters(steps1 - steps0, eps1 - eps0, elapsed, device=red_dev,
                                                    force=args.dist)
    (total_maps,) = reduce_sum([maps1 - maps0], device=red_dev, force=args.dist)
    collective = {"backend": dist.get_backend() if use_dist else None, "executed": use_dist,
                  "device_tensors": bool(use_dist and red_dev is not None), "world": world}
    value = total_steps / t_max

    if args.digest:
        import numpy as np

        from pgtg_amd.digest import Digest
        del actions
        dg = Digest(env)
        t_end = args.warmup + args.steps
        rows = []
        for k in range(args.digest_steps):
            env.step_random(act_seed, t_end + k, env_offset=shard.offset)
            rows.append(dg.step_digest())
        d = torch.stack(rows).cpu().numpy().view(np.uint64)
        np.savez(f"{args.digest}.rank{rank}.npz", digest=d, offset=shard.offset, world=world,
                 steps=t_end, workload=args.workload)

    if rank == 0:
        resets_per_launch = (eps1 - eps0) / max(1, args.steps)
        avg_kernel_s = (kern_ms / max(1, launches)) / 1e3
        cars = env.mean_cars() if spec.traffic_density > 0 else 0.0
        alg = algorithmic_bytes(spec, n_local, resets_per_launch, cars)
        achieved = alg / avg_kernel_s / 1e9 if avg_kernel_s > 0 else 0.0
        peak = max(peak_copy, PEAK_HBM_GUIDE_GBS)  # the higher of the two measured copy rates
        traffic, traffic_src = load_traffic(args.workload, n_local)
        rec = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * t_max / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (device uniform random actions of the global env index, seeds = global env index)",
            "config": {"workload": (f"configs[{cfg_idx}]: " if cfg_idx is not None else "caller: ") + desc,
                       "envs_total": n_total, "envs_per_gpu": n_local,
                       "map": f"{spec.width}x{spec.height}", "traffic_density": spec.traffic_density,
                       "autoreset": True, "parallelism": f"dp{world} (env shards, no data-path collective)"},
            "episodes": total_eps, "collective": collective,
            # k_envq: maps its helper waves generated in the window for later episodes (the rings start
            # full: reset fills them, k_qfill), beside the episodes that took a queued map
            "queue_maps_generated": total_maps if maps1 else None,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                         "frac": achieved / peak if peak > 0 else None, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "peak_source": "max(pgtg_measure_hbm stream copy on this box (2 GiB, read+write bytes), "
                                        "MI355X_MICROARCH.md measured float4 copy 6290 GB/s)",
                         "peak_copy_measured": peak_copy,
                         "peak_spec": PEAK_HBM_SPEC_GBS, "frac_spec": achieved / PEAK_HBM_SPEC_GBS,
                         "kernel": env.step_kernel() + " (step + in-kernel auto-reset)"
                                   + (" + k_traffic (initial traffic of the reset envs)" if spec.traffic_density > 0 else ""),
                         "avg_kernel_us": avg_kernel_s * 1e6, "timed_launches": launches,
                         "kernel_timing": ("HIP event pair around the timed window on the launch stream / launches"
                                           + (": device time per step, both kernels" if spec.traffic_density > 0 else "")
                                           + ("; one host call per step (--per-step): launch gaps included"
                                              if args.per_step else "")),
                         "alg_bytes_per_launch": alg, "alg_model": "SURVEY.md 8(d)",
                         "resets_per_launch": resets_per_launch, "cars_per_env": cars,
                         "envs_per_workgroup": env.launch_info()[0], "lds_bytes": env.launch_info()[1],
                         "workgroups_per_cu": env.occupancy()},
        }
        issue = load_issue(args.workload, n_local, avg_kernel_s)
        if issue is not None:
            rec["roofline_issue"] = issue
        lat = load_latency(args.workload, n_local, avg_kernel_s)
        if lat is not None:
            rec["roofline_latency"] = lat
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(spec, args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    env.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
