"""Container-only loader for the reference (never used on the GPU box, never imported by the
product).  Puts the stand-ins of tools/refshim first on sys.path, then the reference package
directory (its modules use top-level imports), and disables bytecode writing so the read-only
reference tree stays untouched."""
import os
import sys

REF = "/root/reference"
_HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    sys.dont_write_bytecode = True
    for p in (REF, os.path.join(REF, "pgtg"), os.path.join(_HERE, "refshim")):
        if p in sys.path:
            sys.path.remove(p)
        sys.path.insert(0, p)
    import environment  # noqa: E402  (reference pgtg/environment.py)
    import map_generator  # noqa: E402
    import parser as ref_parser  # noqa: E402
    import map as ref_map  # noqa: E402
    import map_tiles_data  # noqa: E402
    import constants  # noqa: E402
    return environment, map_generator, ref_parser, ref_map, map_tiles_data, constants
