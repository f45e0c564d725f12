"""Diagnostic: per-phase wave cycles of k_env from the -DPGTG_STAMPS build (not the product).

Build: hipcc <pgtg_amd.build.FLAGS> -DPGTG_STAMPS -o pgtg_amd/libpgtg_hip_stamps.so pgtg_amd/csrc/pgtg_env.hip
Usage: python tools/stamps.py [cfg2|cfg5|cfg3 ...]
Only waves holding env lanes are summarised; a sub-phase is averaged over the waves whose lane 0
executed it in the last launch (its stamps lie inside that wave's launch window)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pgtg_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.environ.get("PGTG_STAMPS_LIB") or os.path.join(os.path.dirname(_abi.LIB_PATH), "libpgtg_hip_stamps.so")
from pgtg_amd.vector import PGTGVecEnv  # noqa: E402

SLOTS = 32
PHASES = ["stage", "step", "final", "reset", "store", "obs"]
SUB = {"cars": (16, 17), "braking": (17, 18), "reset.seed": (8, 9), "reset.generate": (9, 10),
       "reset.compile": (10, 11), "path.masks": (10, 24), "path.bfs": (24, 25), "path.walk": (25, 11), "reset.start": (11, 12), "gen.start_goal": (9, 13), "gen.edge_init": (13, 14),
       "gen.removal": (14, 15), "gen.tiles": (15, 10), "traf.spawners": (19, 20), "traf.floyd": (20, 21),
       "traf.shuffle": (21, 22), "traf.lookup": (22, 26), "traf.create": (26, 23),
       "final.build": (2, 28), "final.barrier": (28, 29), "final.write": (29, 3),
       "obs.rebuild": (5, 30), "obs.barrier": (30, 31), "obs.write": (31, 6),
       "q.env_step": (1, 22), "q.outputs": (22, 23), "bo.setup": (23, 19), "bo.channels": (19, 20),
       "bo.finish_nsd": (20, 21),
       "grp.post.shfl": (9, 10), "grp.post.build": (10, 11), "grp.post.tail": (11, 2),
       "obsdiag.enter": (23, 9), "obsdiag.scalars": (9, 10), "obsdiag.plan": (10, 11), "obsdiag.tables": (11, 19),
       "grp.rebuild.shfl": (16, 17), "grp.rebuild.build": (17, 18)}
CASES = {"cfg2": (4096, dict(random_map_width=3, random_map_height=3)),
         "cfg5": (131072, dict(random_map_width=5, random_map_height=5)),
         "cfg5big": (1048576, dict(random_map_width=5, random_map_height=5)),
         "cfg4": (262144, dict(random_map_width=3, random_map_height=3)),
         "cfg3": (65536, dict(random_map_width=5, random_map_height=5, traffic_density=0.5))}
import bench  # noqa: E402  (the caller workload: pgtg/train.py's settings)
CASES["train"] = (bench.WORKLOADS["train"][2], dict(bench.WORKLOADS["train"][3]))
for name in (sys.argv[1:] or ["cfg2", "cfg5"]):
    N, kw = CASES[name]
    env = PGTGVecEnv(N, device=0, **kw)
    E, lds = env.launch_info()
    env.reset(seed=0)
    for k in range(int(os.environ.get("PGTG_STAMP_STEPS", "30"))):
        env.step_random(1, k)
        if os.environ.get("PGTG_STAMP_SYNC") == "1":
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    blocks = (N + E - 1) // E
    nw = blocks * 4
    buf = np.zeros(max(nw * SLOTS, (1 << 20) + 8 * nw), np.uint64)
    _abi.lib().pgtg_read_stamps.argtypes = [C.c_void_p, C.c_uint64]
    _abi.lib().pgtg_read_stamps(buf.ctypes.data, buf.size)
    st = buf[:nw * SLOTS].reshape(nw, SLOTS).astype(np.int64)
    # traffic workgroups spread their env slots over all four waves; otherwise envs fill waves in order
    spread = kw.get("traffic_density", 0) > 0
    active = np.ones(nw, bool) if spread else (np.arange(nw) % 4) * 64 < E
    helper = (np.arange(nw) % 4) * 64 == ((E + 63) // 64) * 64
    active &= st[:, 0] != 0  # (the persistent k_envq: only its grid's workgroups hold stamps)
    sh = st[helper]
    okh = (sh[:, 7] > sh[:, 0]) & (sh[:, 7] - sh[:, 0] < 1e8)
    if okh.any():  # map-queue helper wave (k_envq)
        print(f"  queue helper wave: fills {int((sh[okh, 7] - sh[okh, 1]).mean())} cycles "
              f"(max {int((sh[okh, 7] - sh[okh, 1]).max())}), start {int((sh[okh, 1] - sh[okh, 0]).mean())}; "
              f"generate {int((sh[okh, 10] - sh[okh, 9]).mean()) if False else int((sh[okh, 15] - sh[okh, 14]).mean())} "
              f"(removal, last fill)", flush=True)
        seg = lambda a, b: int((sh[okh, b] - sh[okh, a]).mean())  # noqa: E731
        print(f"  helper fill (last): start/goal {seg(1, 13)} (incl. seed pool, child stream), removal {seg(14, 15)} "
              f"(iterations {round(float(sh[okh, 27].mean()), 1)}, max {int(sh[okh, 27].max())}; connectivity tests "
              f"{int(sh[okh, 26].mean())} cycles), borders+obstacles+masks {seg(15, 24)}, path bfs {seg(24, 25)}, "
              f"walk+start+entry {seg(25, 7)}", flush=True)
    st = st[active]
    d = np.diff(st[:, :7], axis=1)
    print(f"{name}: {N} envs, {E} envs/workgroup, LDS {lds} B; cycles per active wave (last launch)", flush=True)
    print("  phases:", {n: int(x) for n, x in zip(PHASES, d.mean(0))}, "total", int((st[:, 6] - st[:, 0]).mean()))
    if os.environ.get("PGTG_STAMPS_JSON"):  # the latency record bench.py reads (profiles/stamps_<workload>.json)
        import json
        tot = st[:, 6] - st[:, 0]
        rec = {"workload": os.environ.get("PGTG_STAMPS_WL", name), "envs": N, "envs_per_workgroup": E,
               "source": "tools/stamps.py (-DPGTG_STAMPS build, s_memtime per wave, last of 30 launches)",
               "wave_chain_cycles_mean": int(tot.mean()), "wave_chain_cycles_p90": int(np.percentile(tot, 90)),
               "wave_chain_cycles_max": int(tot.max()),
               "phases_mean_cycles": {n: int(x) for n, x in zip(PHASES, d.mean(0))}}
        if okh.any():
            rec["helper_fill_cycles_mean"] = int((sh[okh, 7] - sh[okh, 1]).mean())
        with open(os.environ["PGTG_STAMPS_JSON"], "w") as f:
            json.dump(rec, f, indent=1)
    print("  phase p90/max:", {n: (int(np.percentile(d[:, k], 90)), int(d[:, k].max())) for k, n in enumerate(PHASES)},
          "total max", int((st[:, 6] - st[:, 0]).max()))
    lo, hi = st[:, 0], st[:, 6]
    out = {}
    for n, (a, b) in SUB.items():
        if n.startswith("traf.") and spread:  # k_traffic (after k_env; 64-lane workgroups share the slot rows)
            ok = (st[:, a] > 0) & (st[:, b] >= st[:, a]) & (st[:, b] - st[:, a] < 1e9)
        else:
            ok = (st[:, a] >= lo) & (st[:, a] <= hi) & (st[:, b] >= st[:, a]) & (st[:, b] <= hi)
        if ok.any():
            out[n] = (int((st[ok, b] - st[ok, a]).mean()), round(float(ok.mean()), 2))
    print("  sub-phases (mean cycles, fraction of waves):", out, flush=True)
    if spread:  # k_traffic waves: start (slot 27) to end (slot 24), start spread over the grid
        ok = (st[:, 27] > 0) & (st[:, 24] > st[:, 27]) & (st[:, 24] - st[:, 27] < 1e9)
        if ok.any():
            tot = st[ok, 24] - st[ok, 27]
            t0 = st[ok, 27] - st[ok, 27].min()
            pro = st[ok, 19] - st[ok, 27]
            epi = st[ok, 24] - st[ok, 23]
            body = st[ok, 23] - st[ok, 19]
            q = lambda a: (int(a.mean()), int(np.percentile(a, 90)), int(a.max()))  # noqa: E731
            rt = buf[1 << 20:(1 << 20) + 8 * nw].reshape(nw, 8).astype(np.int64)
            e_end, t_beg = rt[:, 0], rt[rt[:, 1] > 0, 1]
            print("  wall clock (10 ns ticks): k_env waves end", 0, "..", int(e_end.max() - e_end.min()),
                  "; k_traffic waves start", int(t_beg.min() - e_end.min()), "..", int(t_beg.max() - e_end.min()), flush=True)
            dv = st[ok, 15]  # the last launch's shape (k_traffic writes it over k_env's slot)
            print("  k_traffic (last launch): list", int(dv[0] & 0xffffffff), "rounds", int((dv[0] >> 32) & 255),
                  "envs per wave", int((dv[0] >> 40) & 255), "LDS capacity per wave", int((dv[0] >> 48) & 255),
                  "(the traffic_reset stamps are the last round's)", flush=True)
            print("  k_traffic waves (mean, p90, max): total", q(tot), "before the last round", q(pro),
                  "last round's traffic_reset", q(body), "epilogue", q(epi), flush=True)
    rt = buf[1 << 20:(1 << 20) + 8 * nw].reshape(nw, 8).astype(np.int64)
    okw = (rt[:, 2] > 0) & (rt[:, 3] > rt[:, 2])
    if not spread and okw.any():  # k_envq: wall-clock start and end of every wave (10 ns ticks, one clock)
        wid = np.arange(nw)[okw]
        t0 = rt[okw, 2].min()
        beg, end = rt[okw, 2] - t0, rt[okw, 3] - t0
        hw = (wid % 4) * 64 == ((E + 63) // 64) * 64
        ew = (wid % 4) * 64 < E
        q = lambda a: (int(a.mean()), int(np.percentile(a, 50)), int(np.percentile(a, 90)), int(a.max()))  # noqa: E731
        print("  wall clock (10 ns ticks from the first wave's start; mean, p50, p90, max): wave starts", q(beg),
              "env-wave ends", q(end[ew]) if ew.any() else None, "helper ends", q(end[hw]) if hw.any() else None,
              "writer-wave ends", q(end[~ew & ~hw]) if (~ew & ~hw).any() else None, flush=True)
    if not spread:  # k_envq env waves: the observation channel loop's split (slots 24, 25)
        okc = (st[:, 24] > 0) & (st[:, 24] < 1e7) & (st[:, 25] < 1e7)
        if okc.any():
            print("  channel loop: code+select", int(st[okc, 24].mean()), "bit sink", int(st[okc, 25].mean()), flush=True)
    # slot 26 is k_traffic's lookup stamp when there is traffic
    okr = (not spread) & (st[:, 14] >= lo) & (st[:, 14] <= hi) & (st[:, 27] > 0) & (st[:, 27] < 1000)
    if okr.any():
        print("  removal loop (lane 0): iterations", round(float(st[okr, 27].mean()), 1), "max", int(st[okr, 27].max()),
              "connectivity-test cycles", int(st[okr, 26].mean()), flush=True)
    env.close()
