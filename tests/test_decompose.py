"""The decomposition restatement against the reference's known answers
(tests/test_environment.py:1126-1151) and its invariants for every |v| <= 64 (CPU)."""
import decompose_ref as dr


def test_reference_known_answers():
    assert dr.decompose(3, 0) == [(1, 0)] * 3
    assert dr.decompose(0, 3) == [(0, 1)] * 3
    assert dr.decompose(3, -3) == [(1, -1)] * 3
    assert dr.decompose(3, 1) == [(1, 0), (1, 1), (1, 0)]
    assert dr.decompose(-1, -3) == [(0, -1), (-1, -1), (0, -1)]


def test_invariants_up_to_64():
    for vx in range(-64, 65):
        for vy in range(-64, 65):
            parts = dr.decompose(vx, vy)
            assert len(parts) == max(abs(vx), abs(vy))
            assert sum(p[0] for p in parts) == vx and sum(p[1] for p in parts) == vy
            assert all(abs(p[0]) <= 1 and abs(p[1]) <= 1 for p in parts)


def test_half_way_rounding_cases_present():
    """|v| >= 10 includes i*m + 0.5 landing exactly on or near an integer, where an FMA or a
    different rounding would change the part (hard part 4)."""
    hits = 0
    for dx in range(10, 65):
        for dy in range(1, dx):
            for i in range(1, dx + 1):
                if (2 * i * dy) % (2 * dx) == dx:  # exact .5
                    hits += 1
    assert hits > 100
