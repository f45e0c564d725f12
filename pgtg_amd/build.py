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
    if force or needs_build():
        cmd = [HIPCC, *FLAGS, "-o", OUT, SRC]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(OUT)
