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
