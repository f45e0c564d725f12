"""CPU oracle's numpy Generator restatement vs numpy itself and vs the committed numpy vectors."""
import ctypes as C
import os

import numpy as np
import pytest

import helpers
from oracle import oracle as O


def _gen(seed, key):
    g = O.OrcPcg()
    O.lib().orc_pcg64_from_seed(int(seed), int(key), 1, C.byref(g))
    return g


def test_seed_sequence_children_match_committed_vectors():
    z = np.load(os.path.join(helpers.GOLDEN, "rng_numpy.npz"))
    for a, s in enumerate(z["seeds"]):
        for b, k in enumerate(z["keys"]):
            g = _gen(s, k)
            st = z["pcg_state"][a, b]
            assert (g.st_hi, g.st_lo, g.inc_hi, g.inc_lo) == tuple(int(x) for x in st)
            raw = [O.lib().orc_next64(C.byref(g)) for _ in range(8)]
            assert raw == [int(x) for x in z["pcg_raw"][a, b]]


def test_mixed_draw_script_matches_committed_vectors():
    z = np.load(os.path.join(helpers.GOLDEN, "rng_numpy.npz"))
    g = _gen(42, 3)
    L = O.lib()
    p = np.array([0.25, 0.35, 0.2, 0.15, 0.05])
    for (kind, n), want in zip(z["script"], z["script_vals"]):
        if kind == 0:
            got = L.orc_random(C.byref(g))
        elif kind == 1:
            got = float(L.orc_integers(C.byref(g), 0, int(n)))
        elif kind == 2:
            got = float(L.orc_choice_p(C.byref(g), p.ctypes.data_as(C.POINTER(C.c_double)), 5))
        else:
            got = float(L.orc_integers(C.byref(g), 1, 4))
        assert got == want


def test_choice_without_replacement_matches_committed_vectors():
    z = np.load(os.path.join(helpers.GOLDEN, "rng_numpy.npz"))
    g = _gen(9, 1)
    flat, i = z["noreplace"], 0
    while i < len(flat):
        pop, k = int(flat[i]), int(flat[i + 1])
        want = flat[i + 2:i + 2 + k]
        out = (C.c_int64 * k)()
        O.lib().orc_choice_noreplace(C.byref(g), pop, k, out)
        assert list(out) == [int(x) for x in want], (pop, k)
        i += 2 + k


@pytest.mark.parametrize("seed", [0, 5, 2**40 + 3])
def test_live_numpy_generator(seed):
    g = _gen(seed, 7)
    ref = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed, spawn_key=(7,))))
    L = O.lib()
    for t in range(500):
        if t % 3 == 0:
            assert L.orc_random(C.byref(g)) == ref.random()
        elif t % 3 == 1:
            n = 2 + t % 97
            assert L.orc_integers(C.byref(g), 0, n) == ref.integers(0, n)
        else:
            assert L.orc_integers(C.byref(g), 0, 9) == ref.choice(9)
