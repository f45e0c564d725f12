"""FlattenObservation layout (pgtg/train.py:40) of batched observations, against a numpy
restatement of gymnasium's flatten for the PGTG Dict space (CPU, synthetic tensors)."""
import warnings

import numpy as np
import pytest
import torch

from pgtg_amd import config as cfg
from pgtg_amd.flat import flat_dim, flat_layout, flatten_obs


def _gym_flatten(obs_i: dict, spec) -> np.ndarray:
    """gymnasium.spaces.flatten on Dict(sorted keys) of the reference's observation space."""
    out = []
    space_keys = sorted(["map", "position", "velocity"] + (["next_subgoal_direction"] if spec.next_subgoal else []))
    for key in space_keys:
        if key == "map":
            for f in sorted(obs_i["map"]):  # inner Dict: sorted feature names, MultiBinary row-major
                out.append(np.asarray(obs_i["map"][f], dtype=np.int8).flatten())
        elif key == "next_subgoal_direction":  # Discrete(9, start=-1)
            oh = np.zeros(9)
            oh[obs_i[key] + 1] = 1
            out.append(oh)
        elif key == "position":  # MultiDiscrete([9, 9])
            oh = np.zeros(18)
            oh[[obs_i[key][0], 9 + obs_i[key][1]]] = 1
            out.append(oh)
        else:  # Box int32 (2,)
            out.append(np.asarray(obs_i[key], dtype=np.int32))
    return np.concatenate([o.astype(np.float64) for o in out])


@pytest.mark.parametrize("kw", [dict(), dict(use_next_subgoal_direction=True),
                                dict(use_sliding_observation_window=True, sliding_observation_window_size=5,
                                     use_next_subgoal_direction=True,
                                     features_to_include_in_observation=["walls", "goals", "traffic", "ice"])])
def test_flatten_matches_gymnasium_order(kw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        spec = cfg.make_spec(**kw)
    N, w = 7, spec.window
    g = torch.Generator().manual_seed(0)
    keys = [k for k, _ in spec.channels]
    obs = {"map": {k: torch.randint(0, 2, (N, w, w), generator=g, dtype=torch.uint8) for k in keys},
           "position": torch.randint(0, 9, (N, 2), generator=g, dtype=torch.int32),
           "velocity": torch.randint(-20, 21, (N, 2), generator=g, dtype=torch.int32)}
    if spec.next_subgoal:
        obs["next_subgoal_direction"] = torch.randint(-1, 8, (N,), generator=g, dtype=torch.int32)
    flat = flatten_obs(spec, obs).numpy()
    assert flat.shape == (N, flat_dim(spec)) == (N, sum(wd for _, wd in flat_layout(spec)))
    for i in range(N):
        oi = {"map": {k: obs["map"][k][i].numpy() for k in keys}, "position": obs["position"][i].numpy(),
              "velocity": obs["velocity"][i].numpy()}
        if spec.next_subgoal:
            oi["next_subgoal_direction"] = int(obs["next_subgoal_direction"][i])
        assert np.array_equal(flat[i], _gym_flatten(oi, spec))


@pytest.mark.parametrize("size", [5, 8, 9, 12])
def test_sliding_position_offsets(size):
    """position (s, s) of a sliding window (environment.py:1453) under MultiDiscrete([9, 9])'s flatten:
    ones at s and 9 + s while they fit the 18 entries; gymnasium's assignment raises IndexError past
    them (s >= 9), so does flatten_obs (no clamping)."""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        spec = cfg.make_spec(use_sliding_observation_window=True, sliding_observation_window_size=size)
    N, w = 3, spec.window
    obs = {"map": {k: torch.zeros((N, w, w), dtype=torch.uint8) for k, _ in spec.channels},
           "position": torch.full((N, 2), size, dtype=torch.int32),
           "velocity": torch.zeros((N, 2), dtype=torch.int32)}
    if size >= 9:
        with pytest.raises(IndexError):
            flatten_obs(spec, obs)
        oh = np.zeros(18)
        with pytest.raises(IndexError):  # numpy's behaviour on gymnasium's offsets + x
            oh[np.array([0, 9]) + np.array([size, size])] = 1
        return
    flat = flatten_obs(spec, obs).numpy()
    pos = flat[:, -20:-2]
    assert (pos.sum(1) == 2).all() and (pos[:, size] == 1).all() and (pos[:, 9 + size] == 1).all()
    oi = {"map": {k: obs["map"][k][0].numpy() for k, _ in spec.channels}, "position": obs["position"][0].numpy(),
          "velocity": obs["velocity"][0].numpy()}
    assert np.array_equal(flat[0], _gym_flatten(oi, spec))
