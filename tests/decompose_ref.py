"""Restatement of PGTGEnv._decompose_velocity (pgtg/environment.py:693-748) and _round (:29-30) in
numpy float64 -- the reference's own arithmetic (Python float = IEEE binary64, `i * m` rounded, then
`+ 0.5`, then floor: no fused multiply-add).  Test infrastructure: the parts a velocity decomposes
into, used by tests/test_decompose.py (pinned to the reference's known answers) and
tests/test_gpu_velocity.py (the GPU's positions after one step)."""
import numpy as np


def _round(x):
    return int(np.floor(x + 0.5))


def decompose(dx: int, dy: int) -> list[tuple[int, int]]:
    if dx == 0 and dy == 0:
        return []
    res = []
    if dx == 0:
        m = int(np.sign(dy))
        res = [(0, i * m) for i in range(1, abs(dy) + 1)]
    elif dy == 0:
        m = int(np.sign(dx))
        res = [(i * m, 0) for i in range(1, abs(dx) + 1)]
    elif abs(dx) >= abs(dy):
        m_y = np.float64(dy) / np.float64(abs(dx))
        m_x = int(np.sign(dx))
        res = [(int(i * m_x), _round(np.float64(i) * m_y)) for i in range(1, abs(dx) + 1)]
    else:
        m_x = np.float64(dx) / np.float64(abs(dy))
        m_y = int(np.sign(dy))
        res = [(_round(np.float64(i) * m_x), int(i * m_y)) for i in range(1, abs(dy) + 1)]
    out, pre = [], (0, 0)
    for v in res:
        out.append((v[0] - pre[0], v[1] - pre[1]))
        pre = v
    return out
