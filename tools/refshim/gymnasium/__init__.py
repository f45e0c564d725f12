"""Minimal stand-in for gymnasium 0.28.1 (poetry.lock pin), used ONLY by tools/gen_golden.py
to import the reference in this container.  Only what the reference touches is provided:
`Env` (lazy `np_random`, seeded `reset`), `spaces.*` (inert), `envs.registration.register`.
Seeding follows gymnasium.utils.seeding.np_random: Generator(PCG64(SeedSequence(seed)))."""
import numpy as np

from . import spaces  # noqa: F401
from .envs import registration  # noqa: F401


class Env:
    _np_random = None
    metadata = {}

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(None)))
        return self._np_random

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            if not (isinstance(seed, int) and seed >= 0):
                raise ValueError("seed must be a non-negative int")
            self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
