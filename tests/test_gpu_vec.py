"""Vector-env features beyond the golden replays: in-kernel TimeLimit truncation (pgtg/train.py:39)
and the SB3 VecEnv adapter with FlattenObservation vectors (pgtg/train.py:40,54), against the
CPU oracle driven the way the wrappers drive the reference."""
import warnings

import numpy as np
import pytest
import torch

import helpers  # noqa: F401
from oracle.oracle import OracleEnv
from pgtg_amd import config as cfg
from pgtg_amd.flat import flatten_obs

pytestmark = pytest.mark.gpu


def _spec(**kw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return cfg.make_spec(**kw)


def _oracle_obs_dict(spec, r):
    keys = [k for k, _ in spec.channels]
    o = {"map": {k: torch.as_tensor(r["obs"][c][None]) for c, k in enumerate(keys)},
         "position": torch.as_tensor(np.array([r["pos"]], np.int32)),
         "velocity": torch.as_tensor(np.array([r["vel"]], np.int32))}
    if spec.next_subgoal:
        o["next_subgoal_direction"] = torch.as_tensor(np.array([r["nsd"]], np.int32))
    return o


def test_time_limit_truncates_and_resets_in_kernel():
    from pgtg_amd.vector import PGTGVecEnv
    spec = _spec(random_map_width=3, random_map_height=3, use_next_subgoal_direction=True)
    N, L = 12, 5
    vec = PGTGVecEnv(N, spec=spec, autoreset=True, max_episode_steps=L)
    vec.reset(seed=40)
    orcs = [OracleEnv(spec) for _ in range(N)]
    for i, o in enumerate(orcs):
        o.reset(40 + i)
    elapsed = np.zeros(N, int)
    rng = np.random.default_rng(5)
    truncs = 0
    for t in range(3 * L):
        acts = np.where(rng.random(N) < 0.8, 4, rng.integers(0, 9, N)).astype(np.uint8)  # mostly stand still
        vec.step(torch.as_tensor(acts))
        torch.cuda.synchronize()
        term, trunc = vec.terminated.cpu().numpy(), vec.truncated.cpu().numpy()
        m, fm = vec.obs_map.cpu().numpy(), vec.final_map.cpu().numpy()
        for i in range(N):
            r = orcs[i].step(int(acts[i]))
            elapsed[i] += 1
            want_trunc = elapsed[i] >= L  # TimeLimit: truncated when the step budget is used up
            assert bool(term[i]) == r["terminated"], (t, i)
            assert bool(trunc[i]) == want_trunc, (t, i)
            if term[i] or trunc[i]:
                assert np.array_equal(fm[i], r["obs"]), (t, i)
                r = orcs[i].reset(None)
                elapsed[i] = 0
                truncs += int(trunc[i])
            assert np.array_equal(m[i], r["obs"]), (t, i)
    assert truncs > 0
    vec.close()


def test_sb3_adapter_flattened_obs_and_terminal_infos():
    from pgtg_amd.sb3 import PGTGSB3VecEnv
    kw = dict(random_map_width=3, random_map_height=3, use_next_subgoal_direction=True)
    spec = _spec(**kw)
    N, L = 8, 6
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        env = PGTGSB3VecEnv(N, max_episode_steps=L, seed=70, **kw)
    obs = env.reset()
    orcs = [OracleEnv(spec) for _ in range(N)]
    rs = [o.reset(70 + i) for i, o in enumerate(orcs)]
    for i in range(N):
        assert np.array_equal(obs[i], flatten_obs(spec, _oracle_obs_dict(spec, rs[i])).numpy()[0])
    elapsed = np.zeros(N, int)
    rng = np.random.default_rng(9)
    seen_done = 0
    for t in range(20):
        acts = rng.integers(0, 9, N)
        obs, rew, dones, infos = env.step(acts)
        assert len(infos) == N and list(infos.finished()) == list(np.nonzero(dones)[0])
        for i in range(N):
            r = orcs[i].step(int(acts[i]))
            elapsed[i] += 1
            assert np.float32(r["reward"]) == rew[i]
            done = r["terminated"] or elapsed[i] >= L
            assert bool(dones[i]) == done, (t, i)
            if done:
                term_flat = flatten_obs(spec, _oracle_obs_dict(spec, r)).numpy()[0]
                assert np.array_equal(infos[i]["terminal_observation"], term_flat)
                assert infos[i]["TimeLimit.truncated"] == (not r["terminated"])
                r = orcs[i].reset(None)
                elapsed[i] = 0
                seen_done += 1
            else:
                assert infos[i] == {}
            assert np.array_equal(obs[i], flatten_obs(spec, _oracle_obs_dict(spec, r)).numpy()[0]), (t, i)
    assert seen_done > 0
    env.close()


def test_sb3_adapter_device_path_equals_host_path():
    """device_obs=True (pgtg_amd/sb3.py): the same flattened observations, rewards, dones and terminal
    observations as the host path, as device tensors, with device actions; SB3's per-env infos on
    demand.  The caller workload's settings (pgtg/train.py:21-40) on 64 envs."""
    from pgtg_amd.sb3 import PGTGSB3VecEnv
    kw = dict(random_map_width=4, random_map_height=4, random_map_obstacle_probability=0.2,
              random_map_percentage_of_connections=0.8, traffic_density=0.2, use_sliding_observation_window=True,
              sliding_observation_window_size=5, use_next_subgoal_direction=True)
    N, L = 64, 7
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        host = PGTGSB3VecEnv(N, max_episode_steps=L, seed=3, **kw)
        dev = PGTGSB3VecEnv(N, max_episode_steps=L, seed=3, device_obs=True, **kw)
    o_h, o_d = host.reset(), dev.reset()
    assert isinstance(o_d, torch.Tensor) and o_d.is_cuda and np.array_equal(o_h, o_d.cpu().numpy())
    g = torch.Generator(device="cuda").manual_seed(1)
    finished = 0
    for t in range(25):
        a = torch.randint(0, 9, (N,), device="cuda", dtype=torch.int64, generator=g)
        o_h, r_h, d_h, i_h = host.step(a.cpu().numpy())
        o_d, r_d, d_d, i_d = dev.step(a)
        assert o_d.is_cuda and r_d.is_cuda and d_d.is_cuda
        assert np.array_equal(o_h, o_d.cpu().numpy()), t
        assert np.array_equal(r_h, r_d.cpu().numpy()) and np.array_equal(d_h, d_d.cpu().numpy()), t
        term = i_d.terminal_observation.cpu().numpy()
        for i in np.nonzero(d_h)[0]:
            assert np.array_equal(i_h[i]["terminal_observation"], term[i])
            assert i_d[i]["TimeLimit.truncated"] == i_h[i]["TimeLimit.truncated"]
            finished += 1
    assert finished > 0
    host.close()
    dev.close()


def test_sharded_batch_equals_the_global_batch():
    """bench/dist sharding: rank r's envs are seeded with r*n_local + i, so two half batches step
    exactly like the global batch (pgtg_amd/dist.py)."""
    from pgtg_amd.dist import Shard
    from pgtg_amd.vector import PGTGVecEnv
    spec = _spec(random_map_width=3, random_map_height=3, traffic_density=0.2)
    n = 32
    full = PGTGVecEnv(2 * n, spec=spec)
    full.reset(seed=0)
    halves = []
    for r in range(2):
        h = PGTGVecEnv(n, spec=spec)
        h.reset(seed=Shard(r, 2, n).offset)
        halves.append(h)
    rng = np.random.default_rng(2)
    for t in range(25):
        a = torch.as_tensor(rng.integers(0, 9, 2 * n).astype(np.uint8))
        full.step(a)
        for r, h in enumerate(halves):
            h.step(a[r * n:(r + 1) * n])
        torch.cuda.synchronize()
        for r, h in enumerate(halves):
            assert torch.equal(full.obs_map[r * n:(r + 1) * n], h.obs_map), (t, r)
            assert torch.equal(full.reward[r * n:(r + 1) * n], h.reward), (t, r)
    for i in (0, n - 1, n, 2 * n - 1):
        assert np.array_equal(full.cars(i), halves[i // n].cars(i % n))


@pytest.mark.parametrize("n,kw,want", [
    (65536, dict(random_map_width=5, random_map_height=5, traffic_density=0.5), 256),  # configs[2]
    (1048576, dict(random_map_width=5, random_map_height=5), 512),                      # configs[4]
    (262144, dict(random_map_width=3, random_map_height=3), 1024),                      # configs[3]
])
def test_step_kernel_occupancy(n, kw, want):
    """The LDS sizing of the bench workloads keeps the intended env lanes per CU resident (envs per
    workgroup x resident workgroups; a few bytes over the budget once halved cfg3's throughput)."""
    from pgtg_amd.vector import PGTGVecEnv
    vec = PGTGVecEnv(n, spec=_spec(**kw))
    try:
        assert vec.launch_info()[0] * vec.occupancy() >= want, (vec.launch_info(), vec.occupancy())
    finally:
        vec.close()


_FLAT_LAYOUTS = {
    # the caller's settings (pgtg/train.py:21-40): D = 1 118, rows of one pass, next-subgoal one-hot
    "caller": dict(random_map_width=4, random_map_height=4, random_map_obstacle_probability=0.2,
                   random_map_percentage_of_connections=0.8, traffic_density=0.2, use_sliding_observation_window=True,
                   sliding_observation_window_size=5, use_next_subgoal_direction=True),
    # D = 461 (441 observation bytes), no next-subgoal one-hot: the tail starts inside chunk 6
    "window3": dict(random_map_width=3, random_map_height=3, traffic_density=0.1, use_sliding_observation_window=True,
                    sliding_observation_window_size=3),
    # D = 2 054: rows in passes of 1 152 values (k_flatten<T, false>)
    "window7": dict(random_map_width=3, random_map_height=3, use_sliding_observation_window=True,
                    sliding_observation_window_size=7, use_next_subgoal_direction=True),
}


@pytest.mark.parametrize("layout", list(_FLAT_LAYOUTS))
@pytest.mark.parametrize("dtype", [torch.float32, torch.int8])
def test_flat_rows_kernel_equals_flatten_obs(dtype, layout):
    """k_flatten (include/pgtg.h pgtg_set_flat_outputs: the FlattenObservation rows written inside the
    step) against flatten_obs, gymnasium's layout: every env's row of the observation after reset and
    each of 30 steps, and the terminal rows of the finished envs (the others untouched), with the
    default feature list, whose name order differs from the observation's channel order, over a
    multi-workgroup batch; three row layouts (one pass with and without the next-subgoal one-hot,
    several passes)."""
    from pgtg_amd.flat import flat_dim
    from pgtg_amd.vector import PGTGVecEnv
    spec = _spec(**_FLAT_LAYOUTS[layout])
    assert [k for k, _ in spec.channels] != sorted(k for k, _ in spec.channels)
    N, T = 3000, 30
    env = PGTGVecEnv(N, spec=spec, device=0, autoreset=True, max_episode_steps=7)
    D = flat_dim(spec)
    flat = torch.empty((N, D), dtype=dtype, device="cuda")
    fin = torch.full((N, D), 77, dtype=dtype, device="cuda")
    env.set_flat_outputs(flat, fin)
    env.reset(seed=11)
    assert torch.equal(flat, flatten_obs(spec, env.observation(), dtype=dtype))
    # the per-env scalars of the same pass (pgtg_set_flat_scalars)
    r32, dn, to = (torch.empty(N, dtype=torch.float32, device="cuda"), torch.empty(N, dtype=torch.bool, device="cuda"),
                   torch.empty(N, dtype=torch.bool, device="cuda"))
    env.set_flat_scalars(r32, dn, to)
    g = torch.Generator(device="cuda").manual_seed(4)
    finished = 0
    for t in range(T):
        fin.fill_(77)
        env.step(torch.randint(0, 9, (N,), device="cuda", dtype=torch.uint8, generator=g))
        assert torch.equal(flat, flatten_obs(spec, env.observation(), dtype=dtype)), t
        done = env.terminated | env.truncated
        assert torch.equal(r32, env.reward.to(torch.float32)) and torch.equal(dn, done), t
        assert torch.equal(to, env.truncated & ~env.terminated), t
        want = flatten_obs(spec, env.final_observation(), dtype=dtype)
        assert torch.equal(fin[done], want[done]), t
        assert bool((fin[~done] == 77).all()), t
        finished += int(done.sum())
    assert finished > N
    env.close()


def test_flat_rows_refused_where_gymnasium_raises():
    from pgtg_amd.flat import flat_dim
    from pgtg_amd.vector import PGTGVecEnv
    spec = _spec(random_map_width=3, random_map_height=3, use_sliding_observation_window=True,
                 sliding_observation_window_size=9)
    env = PGTGVecEnv(4, spec=spec, device=0)
    with pytest.raises(IndexError):
        env.set_flat_outputs(torch.empty((4, flat_dim(spec)), device="cuda"))
    env.close()


def test_sb3_device_actions_out_of_range_are_recorded():
    """A device action outside Discrete(9) (e.g. -1 from an int64 policy output) is never mapped onto a
    valid action: the kernel records PGTG_E_INVALID for that env (error_count())."""
    from pgtg_amd import _abi
    from pgtg_amd.sb3 import PGTGSB3VecEnv
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        env = PGTGSB3VecEnv(8, max_episode_steps=5, seed=1, device_obs=True, random_map_width=3, random_map_height=3)
    env.reset()
    a = torch.zeros(8, dtype=torch.int64, device="cuda")
    a[3], a[5] = -1, 9
    env.step(a)
    n, code = env.venv.error_count()
    assert n == 2 and code == _abi.PGTG_E_INVALID
    env.step(torch.full((8,), 4, dtype=torch.int64, device="cuda"))
    assert env.venv.error_count()[0] == 0
    env.close()
