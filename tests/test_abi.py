"""The C-ABI library builds for gfx950, loads, and exports every entry point include/pgtg.h declares
(no compute calls: no GPU here).  The ctypes structs match the header's layout."""
import ctypes as C
import os
import re
import subprocess

import helpers
from pgtg_amd import _abi, build


def _header_functions():
    src = open(os.path.join(helpers.ROOT, "include", "pgtg.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|uint64_t|const char\*|float)\s+(pgtg_\w+)\(", src, re.M)))


def test_library_builds_and_exports_header_symbols():
    path = build.build()
    syms = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (pgtg_\w+)", syms))
    declared = _header_functions()
    assert declared, "no functions parsed from include/pgtg.h"
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    assert sorted(_abi.EXPORTED) == declared


def test_library_loads_with_ctypes_signatures():
    L = _abi.lib()
    for name in _abi.EXPORTED:
        assert getattr(L, name).argtypes is not None


def test_struct_layout_matches_header():
    # compile a probe against the real header and compare sizes/offsets with ctypes
    probe = r'''
#include <stdio.h>
#include <stddef.h>
#include "pgtg.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(PgtgConfig), sizeof(PgtgRule), sizeof(PgtgOutputs),
         sizeof(PgtgEnvState), offsetof(PgtgConfig, rules), offsetof(PgtgConfig, fm_start),
         offsetof(PgtgConfig, max_episode_steps), sizeof(PgtgCar));
  return 0;
}'''
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "p.c"), "w").write(probe)
        subprocess.run(["gcc", "-I", os.path.join(helpers.ROOT, "include"), "-o", os.path.join(d, "p"),
                        os.path.join(d, "p.c")], check=True)
        out = subprocess.run([os.path.join(d, "p")], capture_output=True, text=True, check=True).stdout.split()
    got = [int(x) for x in out]
    want = [C.sizeof(_abi.PgtgConfig), C.sizeof(_abi.PgtgRule), C.sizeof(_abi.PgtgOutputs),
            C.sizeof(_abi.PgtgEnvState), _abi.PgtgConfig.rules.offset, _abi.PgtgConfig.fm_start.offset,
            _abi.PgtgConfig.max_episode_steps.offset, C.sizeof(_abi.PgtgCar)]
    assert got == want


def test_create_without_gpu_fails_loudly():
    """No silent fallback: creating a handle here (no GPU) must raise, not emulate on the CPU."""
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from pgtg_amd.vector import PGTGVecEnv
    with pytest.raises(Exception):
        PGTGVecEnv(4, device=0, random_map_width=3, random_map_height=3)
