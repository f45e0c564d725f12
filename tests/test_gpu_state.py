"""Device state round trips and the reference's state API on the GPU:
  * pgtg_dump_state / pgtg_load_state: dump at t, k steps, load, the same k steps -> bit-identical
    outputs (every env's digest, pgtg_amd/digest.py), on the same handle and on a fresh handle;
  * PGTGEnv.set_to_state (environment.py:1301-1342) with the reference test's sequence
    (tests/test_environment.py:1086-1124) and, with traffic, against the oracle's set_to_state for
    the steps that follow;
  * PGTGEnv.light_step (environment.py:1283-1299) leaves the env unchanged;
  * save_map (pgtg/map.py:173-184): the saved JSON loads through map_path and reproduces the episode."""
import warnings

import numpy as np
import pytest
import torch

import helpers  # noqa: F401
from oracle.oracle import OracleEnv
from pgtg_amd import config as cfg

pytestmark = pytest.mark.gpu

CONFIGS = {
    "s3_queue": dict(random_map_width=3, random_map_height=3),
    "traffic": dict(random_map_width=4, random_map_height=4, traffic_density=0.3),
    "obstacles_visited": dict(random_map_width=4, random_map_height=4, random_map_obstacle_probability=1.0,
                              random_map_ice_probability_weight=1, random_map_broken_road_probability_weight=1,
                              random_map_sand_probability_weight=1, random_map_traffic_light_probability_weight=1,
                              already_visited_position_penalty=0.5, separate_reward_cost=True),
    "fixed_map": dict(map_path=helpers.TESTDATA + "/map_with_all_directions.json"),
}


def _spec(kw):
    kw = dict(kw)
    mp = kw.pop("map_path", None)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return cfg.make_spec(mp, **kw)


def _rollout(env, dg, acts, t0, k):
    out = []
    for t in range(t0, t0 + k):
        env.step_actions(acts[t])
        out.append(dg.step_digest())
    return torch.stack(out).cpu().numpy()


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_dump_load_replays_bit_exactly(name):
    from pgtg_amd.digest import Digest
    from pgtg_amd.vector import PGTGVecEnv
    spec = _spec(CONFIGS[name])
    n, t_dump, k = 3000, 6, 12
    env = PGTGVecEnv(n, spec=spec, device=0)
    env2 = PGTGVecEnv(n, spec=spec, device=0)
    try:
        env.reset(seed=42)
        acts = env.random_actions(t_dump + k, 0x57A7E)
        dg, dg2 = Digest(env), Digest(env2)
        _rollout(env, dg, acts, 0, t_dump)
        blob = env.dump_state()
        first = _rollout(env, dg, acts, t_dump, k)
        env.load_state(blob)
        again = _rollout(env, dg, acts, t_dump, k)
        assert np.array_equal(first, again), f"{name}: replay after load differs at {np.argwhere(first != again)[:5]}"
        env2.load_state(blob)  # a fresh handle of the same shape
        other = _rollout(env2, dg2, acts, t_dump, k)
        assert np.array_equal(first, other), f"{name}: fresh handle differs at {np.argwhere(first != other)[:5]}"
        assert env.counters() == env2.counters()
    finally:
        env.close()
        env2.close()


def test_load_state_rejects_other_shapes():
    from pgtg_amd.vector import PGTGVecEnv
    a = PGTGVecEnv(64, spec=_spec(CONFIGS["s3_queue"]), device=0)
    b = PGTGVecEnv(65, spec=_spec(CONFIGS["s3_queue"]), device=0)
    c = PGTGVecEnv(64, spec=_spec(CONFIGS["traffic"]), device=0)
    # same shape, other semantics: a different obstacle probability / crash penalty
    d = PGTGVecEnv(64, spec=_spec(dict(CONFIGS["s3_queue"], crash_penalty=7)), device=0)
    e = PGTGVecEnv(64, spec=_spec(dict(CONFIGS["s3_queue"], random_map_percentage_of_connections=0.7)), device=0)
    same = PGTGVecEnv(64, spec=_spec(CONFIGS["s3_queue"]), device=0)
    try:
        a.reset(seed=1)
        blob = a.dump_state()
        for other in (b, c, d, e):
            with pytest.raises(ValueError):
                other.load_state(blob)
        with pytest.raises(ValueError):
            a.load_state(blob[:100])
        same.load_state(blob)  # a handle of the same config accepts it
    finally:
        for h in (a, b, c, d, e, same):
            h.close()


@pytest.mark.parametrize("fixture", ["smallest_simple_env", "simple_env", "obstacle_env"])
def test_set_to_state_reference_sequence(fixture):
    """tests/test_environment.py:1086-1124 with the fixtures of :1157-1187."""
    from pgtg_amd.env import PGTGEnv
    kw = {"smallest_simple_env": dict(random_map_width=1, random_map_height=1, random_map_obstacle_probability=0),
          "simple_env": dict(random_map_width=3, random_map_height=3, random_map_obstacle_probability=0),
          "obstacle_env": dict(random_map_width=3, random_map_height=3, traffic_density=0.02,
                               ignore_traffic_collisions=True)}[fixture]
    env = PGTGEnv(**kw)
    env.reset(seed=0)
    for a in (7, 1, 7, 4, 4):
        env.step(a)
    pos, vel, flat = env.position.copy(), env.velocity.copy(), env.flat_tire
    squares = env.squares().copy()
    cars = [(c.id, c.position, c.route, c.driver_profile) for c in env.cars]
    saved = env.get_info()
    env.step(4)
    env.step(4)
    env.set_to_state(saved)
    assert np.array_equal(pos, env.position) and np.array_equal(vel, env.velocity) and flat == env.flat_tire
    assert np.array_equal(squares, env.squares())
    assert [(c.id, c.position, c.route, c.driver_profile) for c in env.cars] == cars
    assert all(c.patience_counter == 0 and c.last_action_delay == 0 for c in env.cars)
    env.close()


def test_set_to_state_then_steps_match_oracle():
    """Traffic env: after set_to_state(saved info) the next steps equal the oracle's, which was put
    into the same state by its own set_to_state (patience reset, next id = last id + 1)."""
    from pgtg_amd.env import PGTGEnv
    spec = _spec(dict(random_map_width=4, random_map_height=4, traffic_density=0.4))
    rng = np.random.default_rng(3)
    for seed in range(4):
        env = PGTGEnv(random_map_width=4, random_map_height=4, traffic_density=0.4)
        orc = OracleEnv(spec)
        env.reset(seed=seed)
        orc.reset(seed)
        term = False
        for _ in range(3):
            _, _, term, _, _ = env.step(4)
            orc.step(4)
            if term:
                break
        if term:  # crashed into a car while standing: set_to_state does not revive an episode
            env.close()
            continue
        saved = env.get_info()
        saved["cars"] = saved["cars"][::2]  # a different car list than the current one
        obs, info = env.set_to_state(saved)
        cars = [(c["id"], c["x"], c["y"], cfg.ROUTES.index(c["route"]), cfg.DRIVER_PROFILES.index(c["driver_profile"]))
                for c in saved["cars"]]
        r = orc.set_to_state(saved["x"], saved["y"], saved["x_velocity"], saved["y_velocity"], saved["flat_tire"], cars)
        assert np.array_equal(env._vec.obs_map[0].cpu().numpy(), r["obs"])
        assert np.array_equal(env._vec.cars(0), orc.cars())
        for t in range(10):
            a = int(rng.integers(0, 9))
            _, rew, term, _, _ = env.step(a)
            r = orc.step(a)
            assert rew == r["reward"] and term == r["terminated"], (seed, t)
            assert np.array_equal(env._vec.obs_map[0].cpu().numpy(), r["obs"]), (seed, t)
            assert np.array_equal(env._vec.cars(0), orc.cars()), (seed, t)
            if term:
                break
        env.close()


def test_light_step_leaves_env_unchanged():
    from pgtg_amd.env import PGTGEnv
    env = PGTGEnv(random_map_width=4, random_map_height=4, traffic_density=0.3, random_map_obstacle_probability=0.5)
    ref = PGTGEnv(random_map_width=4, random_map_height=4, traffic_density=0.3, random_map_obstacle_probability=0.5)
    env.reset(seed=9)
    ref.reset(seed=9)
    for a in (5, 7, 4, 8, 3, 4, 6):
        lo = env.light_step(a)
        o = env.step(a)
        r = ref.step(a)
        for x, y in ((lo, r), (o, r)):
            assert x[1] == y[1] and x[2] == y[2]
            assert np.array_equal(x[0]["map"]["walls"], y[0]["map"]["walls"])
            assert all(np.array_equal(x[0]["map"][k], y[0]["map"][k]) for k in y[0]["map"])
            assert np.array_equal(x[0]["position"], y[0]["position"])
        if o[2]:
            break
    env.close()
    ref.close()


@pytest.mark.parametrize("seed", [0, 5, 17])
def test_save_map_round_trip(tmp_path, seed):
    """The saved map loads through map_path: same squares; after putting the agent on the same square
    the episode continues identically (only map_rng, which draws the start square, differs)."""
    from pgtg_amd.env import PGTGEnv
    kw = dict(random_map_width=4, random_map_height=3, random_map_obstacle_probability=0.6)
    env = PGTGEnv(**kw)
    env.reset(seed=seed)
    p = str(tmp_path / f"m{seed}")
    env.save_map(p)
    fixed = PGTGEnv(p + ".json", random_map_obstacle_probability=0.6)
    fixed.reset(seed=seed)
    assert fixed.map_plan() == env.map_plan()
    st = env.get_info()
    fixed.set_to_state(st)
    s0, s1 = env.squares(), fixed.squares()
    start_bit = np.uint64(1 << 38)
    assert np.array_equal(s0 & ~start_bit, s1 & ~start_bit)
    rng = np.random.default_rng(seed)
    for t in range(15):
        a = int(rng.integers(0, 9))
        x, y = env.step(a), fixed.step(a)
        assert x[1] == y[1] and x[2] == y[2], t
        assert all(np.array_equal(x[0]["map"][k], y[0]["map"][k]) for k in x[0]["map"]), t
        if x[2]:
            break
    env.close()
    fixed.close()


def _sections(a, b):
    """{section id: (bytes of a, bytes of b)} of two pgtg_dump_state blobs (layout: PgtgStateHeader,
    n_sections x {id u32, pad u32, bytes u64}, each section at a 16-byte aligned offset)."""
    hdr = 4 + 4 + 8 + 4 * 4 + 4 * 4 + 8
    n_sec = int(np.frombuffer(a[16:20].tobytes(), np.uint32)[0])
    ent = np.frombuffer(a[hdr:hdr + 16 * n_sec].tobytes(), dtype=[("id", "<u4"), ("pad", "<u4"), ("bytes", "<u8")])
    off, out = hdr + 16 * n_sec, {}
    for e in ent:
        off = (off + 15) & ~15
        out[int(e["id"])] = (a[off:off + int(e["bytes"])], b[off:off + int(e["bytes"])])
        off += int(e["bytes"])
    assert off == a.size, (off, a.size)
    return out


@pytest.mark.parametrize("name", ["s3_queue", "traffic"])
def test_step_many_equals_step_loop(name):
    """pgtg_step_many (one host call for T ticks from a [T, N] buffer) == T pgtg_step calls: the
    same digests after the last tick and on the ticks that follow."""
    from pgtg_amd.digest import Digest
    from pgtg_amd.vector import PGTGVecEnv
    spec = _spec(CONFIGS[name])
    n, k = 3000, 17  # odd k: the traffic handle's car-bank parity flips per launch
    a, b = PGTGVecEnv(n, spec=spec, device=0), PGTGVecEnv(n, spec=spec, device=0)
    try:
        a.reset(seed=7)
        b.reset(seed=7)
        acts = a.random_actions(k, 0x5EED)
        for t in range(k):
            a.step_actions(acts[t])
        b.step_many(acts)
        da, db = Digest(a).step_digest().cpu().numpy(), Digest(b).step_digest().cpu().numpy()
        assert np.array_equal(da, db), f"{name}: digests differ at {np.argwhere(da != db)[:5]}"
        assert a.counters() == b.counters()
        # identical work leaves identical state: every section of the blob (agent records, plans,
        # RNG streams, car slots, spawner lists, map-queue rings and their counts) byte for byte
        sa, sb = a.dump_state(), b.dump_state()
        assert sa.size == sb.size
        diff = [sec for sec, (x, y) in _sections(sa, sb).items() if not np.array_equal(x, y)]
        assert not diff, f"{name}: state sections differ: {diff}"
        more = a.random_actions(8, 0x5EED, t0=k)
        ra, rb = _rollout(a, Digest(a), more, 0, 8), _rollout(b, Digest(b), more, 0, 8)
        assert np.array_equal(ra, rb), f"{name}: later ticks differ at {np.argwhere(ra != rb)[:5]}"
        with pytest.raises(ValueError):
            b.step_many(acts[0])
    finally:
        a.close()
        b.close()


def test_persisted_occupancy_counters_match_cars():
    """The persisted 4-bit lane-square counters match the env's current cars: per tile, the nibble sum
    equals the env's cars on that tile.  traf.w bit 0 = counters exact; bit 1 = fresh traffic, whose
    cars and counters k_traffic wrote to the env's contiguous staging block (blob section 37: w0 of the
    cars, then the counters at fresh_occ), else the counters are DevState::occ's slot-major rows
    (section 36, written by k_env after every unsaturated step).  k_env loads them instead of
    rebuilding them from the car slots; a host car write (add_car / set_to_state) clears the flags."""
    from pgtg_amd.vector import PGTGVecEnv
    spec = _spec(CONFIGS["traffic"])
    n, tw, th = 3000, 4, 4
    nw = tw * th * 4
    env = PGTGVecEnv(n, spec=spec, device=0)

    def counters(sec, i, flags):
        if flags & 2:  # fresh: the staging block
            blk = sec[37][0].view(np.uint32).reshape(n, -1)
            fresh_occ = blk.shape[1] - nw
            words = blk[i, fresh_occ:]
        else:
            words = sec[36][0].view(np.uint32).reshape(nw, n)[:, i]
        words = words.reshape(tw * th, 4)
        return sum(((words >> (4 * b)) & 15).sum(axis=1) for b in range(8))

    try:
        env.reset(seed=5)
        acts = env.random_actions(9, 0x0CC)
        checked, fresh_seen = 0, 0
        for t in range(9):
            env.step_actions(acts[t])
            if t not in (0, 8):
                continue
            blob = env.dump_state()
            sec = _sections(blob, blob)
            traf = sec[34][0].view(np.uint32).reshape(n, 4)
            valid = np.flatnonzero(traf[:, 3] & 1)
            assert valid.size > n // 2, f"t{t}: only {valid.size} envs with persisted counters"
            fresh_seen += int(((traf[:, 3] & 2) != 0).sum())
            for i in valid[:: max(1, valid.size // 200)]:
                nib = counters(sec, int(i), int(traf[i, 3]))
                cars = env.cars(int(i))
                per_tile = np.bincount((cars[:, 2] // 9) * tw + cars[:, 1] // 9, minlength=tw * th)
                assert np.array_equal(nib, per_tile), f"t{t} env {i}: counters {nib} vs cars {per_tile}"
                checked += 1
        assert checked > 300 and fresh_seen > 0
        # a host car write (add_car / set_to_state) invalidates the env's counters; the next step
        # rebuilds them and persists them again
        c0 = env.cars(0)
        env.add_car(0, int(c0[0, 1]), int(c0[0, 2]), int(c0[0, 3]), int(c0[0, 4]))
        sec = _sections(env.dump_state(), env.dump_state())
        assert sec[34][0].view(np.uint32).reshape(n, 4)[0, 3] == 0
        env.step_actions(env.random_actions(1, 0x0CD)[0])
        blob = env.dump_state()
        sec = _sections(blob, blob)
        f0 = int(sec[34][0].view(np.uint32).reshape(n, 4)[0, 3])
        if f0 & 1:
            cars = env.cars(0)
            assert np.array_equal(counters(sec, 0, f0), np.bincount((cars[:, 2] // 9) * tw + cars[:, 1] // 9,
                                                                    minlength=tw * th))
    finally:
        env.close()
