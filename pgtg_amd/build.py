"""Build the in-tree HIP library for gfx950 (and nothing else): `python -m pgtg_amd.build`."""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(PKG, "csrc", "pgtg_env.hip")
DEPS = [SRC, os.path.join(PKG, "csrc", "pgtg_device.h"), os.path.join(PKG, "csrc", "pgtg_tables.h"),
        os.path.join(os.path.dirname(PKG), "include", "pgtg.h")]
OUT = os.path.join(PKG, "libpgtg_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False, verbose: bool = False) -> str:
    """(Re)build the library if a source is newer.  Serialised by a file lock so that the ranks of a
    multi-process run can all call it: one compiles, the others wait and find it up to date."""
    import fcntl
    with open(OUT + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if force or needs_build():
                tmp = OUT + f".tmp{os.getpid()}"
                cmd = [HIPCC, *FLAGS, "-o", tmp, SRC]
                if verbose:
                    print(" ".join(cmd), flush=True)
                subprocess.run(cmd, check=True)
                os.replace(tmp, OUT)  # atomic: a concurrent loader never sees a partial file
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(OUT)
