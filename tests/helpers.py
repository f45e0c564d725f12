"""Shared test helpers: golden-fixture loading and vectorised replay of the CPU oracle."""
from __future__ import annotations

import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
TESTDATA = os.path.join(ROOT, "tests", "golden", "maps")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from pgtg_amd.config import make_spec  # noqa: E402


def load_traj(name: str) -> dict:
    z = np.load(os.path.join(GOLDEN, f"traj_{name}.npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(bytes(d["meta"]).decode())
    return d


def traj_names() -> list[str]:
    return sorted(f[5:-4] for f in os.listdir(GOLDEN) if f.startswith("traj_"))


def spec_for(meta: dict):
    kw = dict(meta["kwargs"])
    for k in ("random_map_start_position", "random_map_goal_position", "traffic_light_phases_duration"):
        if isinstance(kw.get(k), list):
            kw[k] = tuple(kw[k])
    mp = os.path.join(TESTDATA, meta["map_file"]) if meta["map_file"] else None
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return make_spec(mp, **kw)


def digest(arr) -> int:
    return zlib.crc32(np.ascontiguousarray(arr, dtype=np.int32).tobytes())


def channel_perm(spec, keys: list[str]) -> list[int]:
    """index into our channel order for each golden key"""
    ours = [k for k, _ in spec.channels]
    return [ours.index(k) for k in keys]


def replay_oracle(d: dict, n_envs: int | None = None, steps: int | None = None) -> list[str]:
    """Replay the golden trajectory through the CPU oracle; return a list of mismatch strings."""
    from oracle.oracle import OracleEnv
    meta = d["meta"]
    spec = spec_for(meta)
    perm = channel_perm(spec, meta["keys"])
    N = meta["N"] if n_envs is None else min(n_envs, meta["N"])
    T = meta["T"] if steps is None else min(steps, meta["T"])
    reset_map = {(int(t), int(i)): k for k, (t, i) in enumerate(d["reset_idx"])}
    bad: list[str] = []
    for i in range(N):
        env = OracleEnv(spec)
        r = env.reset(meta["seed_base"] + i)
        if not np.array_equal(r["obs"][perm], d["init_obs"][i]):
            bad.append(f"env{i} reset obs")
        if tuple(r["pos"]) != tuple(d["init_pos"][i]):
            bad.append(f"env{i} reset pos")
        if digest(env.cars()) != int(d["init_cars_dig"][i]):
            bad.append(f"env{i} reset cars")
        for t in range(T):
            r = env.step(int(d["actions"][t, i]))
            tag = f"env{i} t{t}"
            if not np.array_equal(r["obs"][perm], d["obs"][t, i]):
                diff = [meta["keys"][c] for c in range(len(perm)) if not np.array_equal(r["obs"][perm[c]], d["obs"][t, i, c])]
                bad.append(f"{tag} obs {diff}")
            if tuple(r["pos"]) != tuple(d["pos"][t, i]) or tuple(r["vel"]) != tuple(d["vel"][t, i]):
                bad.append(f"{tag} pos/vel {r['pos']} {r['vel']} vs {d['pos'][t, i]} {d['vel'][t, i]}")
            if r["reward"] != d["reward"][t, i] or r["cost"] != d["cost"][t, i]:
                bad.append(f"{tag} reward {r['reward']} vs {d['reward'][t, i]}")
            if r["terminated"] != bool(d["terminated"][t, i]):
                bad.append(f"{tag} terminated")
            if spec.next_subgoal and r["nsd"] != d["nsd"][t, i]:
                bad.append(f"{tag} nsd {r['nsd']} vs {d['nsd'][t, i]}")
            if bool(r["braking"]) != bool(d["braking"][t, i]):
                bad.append(f"{tag} braking")
            if digest(env.cars()) != int(d["cars_dig"][t, i]):
                bad.append(f"{tag} cars")
            if r["terminated"]:
                k = reset_map[(t, i)]
                r = env.reset(None)
                if not np.array_equal(r["obs"][perm], d["reset_obs"][k]):
                    bad.append(f"{tag} autoreset obs")
                if tuple(r["pos"]) != tuple(d["reset_pos"][k]):
                    bad.append(f"{tag} autoreset pos")
                if digest(env.cars()) != int(d["reset_cars_dig"][k]):
                    bad.append(f"{tag} autoreset cars")
            if len(bad) > 20:
                return bad
    return bad


def has_traffic(meta: dict) -> bool:
    return float(meta["kwargs"].get("traffic_density", 0) or 0) > 0


def replay_vec(d: dict, n_envs: int | None = None, steps: int | None = None) -> list[str]:
    """Replay a golden trajectory through the HIP vector env (auto-reset); mismatch strings."""
    import torch
    from pgtg_amd.vector import PGTGVecEnv
    meta = d["meta"]
    spec = spec_for(meta)
    perm = channel_perm(spec, meta["keys"])
    N = meta["N"] if n_envs is None else min(n_envs, meta["N"])
    T = meta["T"] if steps is None else min(steps, meta["T"])
    env = PGTGVecEnv(N, spec=spec, autoreset=True)
    bad: list[str] = []
    obs, _ = env.reset(seed=meta["seed_base"])
    torch.cuda.synchronize()
    m = env.obs_map.cpu().numpy()[:, perm]
    pos = env.position.cpu().numpy()
    for i in range(N):
        if has_traffic(meta) and digest(env.cars(i)) != int(d["init_cars_dig"][i]):
            bad.append(f"env{i} reset cars")
        if not np.array_equal(m[i], d["init_obs"][i]):
            bad.append(f"env{i} reset obs")
        if tuple(pos[i]) != tuple(d["init_pos"][i]):
            bad.append(f"env{i} reset pos {pos[i]} vs {d['init_pos'][i]}")
        if spec.next_subgoal and int(env.nsd[i]) != int(d["init_nsd"][i]):
            bad.append(f"env{i} reset nsd")
    reset_map = {(int(t), int(i)): k for k, (t, i) in enumerate(d["reset_idx"])}
    for t in range(T):
        acts = torch.as_tensor(d["actions"][t, :N].astype(np.uint8)).cuda()
        env.step(acts)
        torch.cuda.synchronize()
        m = env.obs_map.cpu().numpy()[:, perm]
        fm = env.final_map.cpu().numpy()[:, perm]
        pos, vel = env.position.cpu().numpy(), env.velocity.cpu().numpy()
        fpos, fvel = env.final_position.cpu().numpy(), env.final_velocity.cpu().numpy()
        rew, term = env.reward.cpu().numpy(), env.terminated.cpu().numpy()
        trunc = env.truncated.cpu().numpy()
        cost = env.cost.cpu().numpy() if env.cost is not None else np.zeros(N)
        brk = env.braking.cpu().numpy()
        nsd = env.nsd.cpu().numpy() if env.nsd is not None else None
        fnsd = env.final_nsd.cpu().numpy() if env.final_nsd is not None else None
        check_cars = has_traffic(meta)
        for i in range(N):
            tag = f"env{i} t{t}"
            if check_cars:
                dig = digest(env.cars(i))
                want = d["reset_cars_dig"][reset_map[(t, i)]] if term[i] else d["cars_dig"][t, i]
                if dig != int(want):
                    bad.append(f"{tag} cars")
            if bool(term[i]) != bool(d["terminated"][t, i]) or trunc[i]:
                bad.append(f"{tag} terminated {term[i]} vs {d['terminated'][t, i]}")
                continue
            if bool(brk[i]) != bool(d["braking"][t, i]):
                bad.append(f"{tag} braking {brk[i]} vs {d['braking'][t, i]}")
            if rew[i] != d["reward"][t, i] or cost[i] != d["cost"][t, i]:
                bad.append(f"{tag} reward {rew[i]} vs {d['reward'][t, i]} cost {cost[i]} vs {d['cost'][t, i]}")
            if term[i]:
                if not np.array_equal(fm[i], d["obs"][t, i]):
                    bad.append(f"{tag} final obs")
                if tuple(fpos[i]) != tuple(d["pos"][t, i]) or tuple(fvel[i]) != tuple(d["vel"][t, i]):
                    bad.append(f"{tag} final pos/vel")
                if fnsd is not None and fnsd[i] != d["nsd"][t, i]:
                    bad.append(f"{tag} final nsd")
                k = reset_map[(t, i)]
                if not np.array_equal(m[i], d["reset_obs"][k]):
                    bad.append(f"{tag} autoreset obs")
                if tuple(pos[i]) != tuple(d["reset_pos"][k]):
                    bad.append(f"{tag} autoreset pos")
                if nsd is not None and nsd[i] != d["reset_nsd"][k]:
                    bad.append(f"{tag} autoreset nsd")
            else:
                if not np.array_equal(m[i], d["obs"][t, i]):
                    diff = [meta["keys"][c] for c in range(len(perm)) if not np.array_equal(m[i, c], d["obs"][t, i, c])]
                    bad.append(f"{tag} obs {diff}")
                if tuple(pos[i]) != tuple(d["pos"][t, i]) or tuple(vel[i]) != tuple(d["vel"][t, i]):
                    bad.append(f"{tag} pos/vel {pos[i]} {vel[i]} vs {d['pos'][t, i]} {d['vel'][t, i]}")
                if nsd is not None and nsd[i] != d["nsd"][t, i]:
                    bad.append(f"{tag} nsd {nsd[i]} vs {d['nsd'][t, i]}")
            if len(bad) > 30:
                env.close()
                return bad
    env.close()
    return bad
