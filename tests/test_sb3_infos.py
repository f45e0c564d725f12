"""The SB3 adapter's lazy per-env infos (pgtg_amd/sb3.py VecInfos): the same dicts SB3's VecEnv
protocol expects (terminal_observation / TimeLimit.truncated for finished envs, cost), built on
read, no GPU needed."""
import numpy as np
import pytest

from pgtg_amd.sb3 import VecInfos


def test_vecinfos_matches_the_eager_list():
    n = 6
    dones = np.array([0, 1, 0, 1, 1, 0], bool)
    trunc = np.array([0, 0, 0, 1, 0, 0], bool)
    final = np.arange(n * 3, dtype=np.float32).reshape(n, 3)
    cost = np.linspace(0, 1, n)
    inf = VecInfos(dones, trunc, final, cost)
    eager = []
    for i in range(n):
        d = {}
        if dones[i]:
            d["terminal_observation"] = final[i]
            d["TimeLimit.truncated"] = bool(trunc[i])
        d["cost"] = float(cost[i])
        eager.append(d)
    assert len(inf) == n
    for a, b in zip(inf, eager):
        assert a.keys() == b.keys()
        for k in a:
            assert np.array_equal(a[k], b[k])
    assert inf[-1] == eager[-1] and len(inf[1:4]) == 3
    assert inf.finished().tolist() == [1, 3, 4]
    with pytest.raises(IndexError):
        inf[n]
    assert VecInfos(np.zeros(3, bool), np.zeros(3, bool), None, None)[2] == {}


def test_vecinfos_entries_persist_in_place_edits():
    """SB3's VecNormalize/VecFrameStack rewrite infos[i]["terminal_observation"] in place and read it
    back: the sequence must hand out the same dict each time."""
    dones = np.array([1, 0, 1], bool)
    final = np.ones((3, 4), np.float32)
    inf = VecInfos(dones, np.zeros(3, bool), final, None)
    x = np.full(4, 7.0, np.float32)
    inf[0]["terminal_observation"] = x
    assert inf[0]["terminal_observation"] is x and inf[0] is inf[0]
    assert inf[:1][0]["terminal_observation"] is x and list(inf)[0] is inf[0]
    inf[-1]["extra"] = 1
    assert inf[2]["extra"] == 1


def test_vecinfos_finished_rows_and_full_reads():
    """Terminal observations stored one row per finished env (final_rows), and VecMonitor's
    list(infos[:]) (pgtg/train.py:55) giving the same dict objects as per-env reads, before and after."""
    dones = np.array([0, 1, 0, 0, 1], bool)
    rows = np.array([-1, 0, -1, -1, 1])
    final = np.array([[1.0, 2.0], [3.0, 4.0]], np.float32)
    cost = np.array([0.5, 0.0, 1.0, 2.0, 0.25])
    inf = VecInfos(dones, np.zeros(5, bool), final, cost, rows)
    first = inf[4]
    allv = list(inf[:])
    assert allv[4] is first and inf[4] is first and inf[1] is allv[1]
    assert np.array_equal(allv[1]["terminal_observation"], final[0]) and np.array_equal(first["terminal_observation"], final[1])
    assert allv[0] == {"cost": 0.5} and allv[3] == {"cost": 2.0} and allv[1]["cost"] == 0.0
    assert len(inf[1:3]) == 2 and inf[-1] is first
