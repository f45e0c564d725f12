"""pgtg_amd -- MI355X-native batched PGTG (ProcGrid Traffic Gym) step/reset.

Drop-in for the reference's hot path (Inuri04/pgtg `PGTGEnv.step/reset`, registered as "pgtg-v4"):
  PGTGVecEnv  -- N independent episodes in lockstep on one GPU (HIP kernels via include/pgtg.h)
  PGTGEnv     -- single-env Gymnasium-style facade with the reference's constructor and returns
"""
from .config import EnvSpec, make_spec  # noqa: F401

__version__ = "0.5.0"  # the reference's pgtg/__init__.py version this build mirrors


def __getattr__(name):
    if name == "PGTGVecEnv":
        from .vector import PGTGVecEnv
        return PGTGVecEnv
    if name == "PGTGEnv":
        from .env import PGTGEnv
        return PGTGEnv
    raise AttributeError(name)


def register_gymnasium() -> bool:
    """Register "pgtg-v4" with gymnasium if it is installed (pgtg/__init__.py:7)."""
    try:
        from gymnasium.envs.registration import register
    except ImportError:
        return False
    register(id="pgtg-v4", entry_point="pgtg_amd.env:PGTGEnv")
    return True
