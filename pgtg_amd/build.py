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


# test variant: occupancy counters saturating at 2 cars so that the exact-recount path runs often
# (tests/test_gpu_occupancy.py replays the traffic trajectories through it)
VARIANTS = {"occsat": ["-DPGTG_OCC_MAX=2"]}
# A/B and diagnostic build (tools/*.sh): reads the PGTG_SPREAD/COMPACT/QUEUE/LINEMASK/DIAG knobs from
# the environment; the product library reads none.  Not built by default (PGTG_LIB selects it).
TOOL_VARIANTS = {"tuning": ["-DPGTG_TUNING"], "stamps": ["-DPGTG_STAMPS"], "ntobs": ["-DPGTG_NT_OBS"],
                 "stampsobs": ["-DPGTG_STAMPS", "-DPGTG_STAMPS_OBS"]}


def variant_path(name: str) -> str:
    return os.path.join(PKG, f"libpgtg_hip_{name}.so")


def needs_build(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False, verbose: bool = False, variant: str | None = None) -> str:
    """(Re)build the library if a source is newer.  Serialised by a file lock so that the ranks of a
    multi-process run can all call it: one compiles, the others wait and find it up to date."""
    import fcntl
    out = OUT if variant is None else variant_path(variant)
    extra = [] if variant is None else {**VARIANTS, **TOOL_VARIANTS}[variant]
    with open(out + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if force or needs_build(out):
                tmp = out + f".tmp{os.getpid()}"
                cmd = [HIPCC, *FLAGS, *extra, "-o", tmp, SRC]
                if verbose:
                    print(" ".join(cmd), flush=True)
                subprocess.run(cmd, check=True)
                os.replace(tmp, out)  # atomic: a concurrent loader never sees a partial file
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return out


def build_all(force: bool = False, verbose: bool = False, variants=tuple(VARIANTS)) -> list[str]:
    """The product library and the given variants, compiled concurrently (one hipcc each)."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=1 + len(variants)) as ex:
        futs = [ex.submit(build, force, verbose, v) for v in (None, *variants)]
        return [f.result() for f in futs]


if __name__ == "__main__":
    tools = [a.split("=", 1)[1].split(",") for a in sys.argv if a.startswith("--tools=")]
    print("\n".join(build_all(force="--force" in sys.argv, verbose=True,
                               variants=tuple(VARIANTS) + tuple(tools[0] if tools else ()))))
