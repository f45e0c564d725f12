#!/usr/bin/env python3
"""Compare the per-env output digests of a sharded bench run with a single-GPU run of the same batch.

    python tools/digest_compare.py <single-prefix> <sharded-prefix>

<prefix>.rank<r>.npz are written by `bench.py --digest <prefix>`.  Every rank's slice
[offset, offset + n_local) must equal the same slice of the single-GPU digests at every step.
Prints one JSON line; exit status 1 on a mismatch.
"""
import glob
import json
import sys

import numpy as np


def load(prefix):
    parts = []
    for f in sorted(glob.glob(prefix + ".rank*.npz")):
        z = np.load(f, allow_pickle=False)
        parts.append((int(z["offset"]), z["digest"], int(z["world"]), int(z["steps"])))
    return sorted(parts, key=lambda p: p[0])


def main():
    single, sharded = load(sys.argv[1]), load(sys.argv[2])
    assert len(single) == 1, "the reference run must have one rank"
    ref = single[0][1]
    rec = {"envs": int(ref.shape[1]), "digest_steps": int(ref.shape[0]), "ranks": len(sharded), "ranks_equal": []}
    ok = len(sharded) == sharded[0][2] if sharded else False
    for off, d, _, steps in sharded:
        eq = d.shape[0] == ref.shape[0] and steps == single[0][3] and np.array_equal(d, ref[:, off:off + d.shape[1]])
        rec["ranks_equal"].append({"offset": off, "envs": int(d.shape[1]), "equal": bool(eq)})
        ok = ok and eq
    covered = sum(d.shape[1] for _, d, _, _ in sharded)
    ok = ok and covered == ref.shape[1]
    rec["all_equal"] = bool(ok)
    print(json.dumps(rec))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
