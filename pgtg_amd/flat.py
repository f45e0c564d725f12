"""FlattenObservation layout of the PGTG observation (pgtg/train.py:39-40) for batched tensors.

gymnasium's `Dict` space orders a plain-dict's keys by name, and `flatten` concatenates its
subspaces in that order: `MultiBinary((w, w))` as the w*w values row-major, `Discrete(n, start)` as a
one-hot of length n at `x - start`, `MultiDiscrete(nvec)` as one one-hot per component, `Box` as its
values.  For the PGTG space (environment.py:415-441) that is

    map/<features sorted by name> (w*w each) | next_subgoal_direction (9, one-hot of d+1) |
    position (9 + 9 one-hots) | velocity (2)

`flatten_obs` builds that vector for every env of a batch from the device tensors of a `PGTGVecEnv`
observation with torch ops (the reference formula the tests compare with); the product path writes
the same rows with the HIP kernel `k_flatten` after every step (`PGTGVecEnv.set_flat_outputs`,
include/pgtg.h `pgtg_set_flat_outputs`).
"""
from __future__ import annotations


def flat_layout(spec) -> list[tuple[str, int]]:
    """(field, width) in gymnasium's flatten order."""
    win = spec.window
    out = [(f"map/{k}", win * win) for k in sorted(k for k, _ in spec.channels)]
    if spec.next_subgoal:
        out.append(("next_subgoal_direction", 9))
    out += [("position", 18), ("velocity", 2)]
    return out


def flat_dim(spec) -> int:
    return sum(w for _, w in flat_layout(spec))


def flat_order(spec) -> list[int]:
    """order[k] = index in spec.channels (the observation's channel order) of the k-th key by name:
    the channel permutation of the device flattener (include/pgtg.h pgtg_set_flat_outputs)."""
    keys = [k for k, _ in spec.channels]
    return sorted(range(len(keys)), key=lambda i: keys[i])


def check_flattenable(spec) -> None:
    """gymnasium's flatten raises for a sliding window of size >= 9 (see flatten_obs)."""
    if spec.sliding and spec.sliding_size >= 9:
        raise IndexError(f"position ({spec.sliding_size}, {spec.sliding_size}) is outside MultiDiscrete([9, 9]): "
                         f"index {9 + spec.sliding_size} is out of bounds for its flattened size 18")


def flatten_obs(spec, obs: dict, dtype=None):
    """obs: a PGTGVecEnv observation dict ({"map": {k: [N, w, w]}, "position": [N, 2], ...}) ->
    [N, flat_dim] tensor (float32 by default) on the same device."""
    import torch
    dtype = torch.float32 if dtype is None else dtype
    pos = obs["position"].long()
    n = pos.shape[0]
    parts = [obs["map"][k].reshape(n, -1).to(dtype) for k in sorted(obs["map"])]
    if spec.next_subgoal:
        parts.append(torch.nn.functional.one_hot(obs["next_subgoal_direction"].long() + 1, 9).to(dtype))
    # MultiDiscrete([9, 9]): one 18-entry vector with ones at offsets + x = (x, 9 + y).  The position is
    # the agent's square in its tile (0..8) or, with a sliding window, (s, s) (environment.py:1453), so
    # a window of size s >= 9 puts 9 + s past the vector's end, where gymnasium's index assignment
    # raises -- as here, decided from the spec without reading the tensor.
    check_flattenable(spec)
    oh = torch.zeros((n, 18), dtype=dtype, device=pos.device)
    oh.scatter_(1, torch.stack([pos[:, 0], 9 + pos[:, 1]], dim=1), 1)
    parts.append(oh)
    parts.append(obs["velocity"].to(dtype))
    return torch.cat(parts, dim=1)
