"""Host-side kwargs handling mirrors the reference's validation and observation-key semantics."""
import math
import warnings

import pytest

from pgtg_amd import config as C


def test_defaults_match_reference_constructor():
    s = C.make_spec()
    assert (s.width, s.height, s.pct_connections) == (4, 4, 0.5)
    assert [k for k, _ in s.channels] == C.DEFAULT_FEATURES
    assert s.window == 9 and len(s.rules) == 2


@pytest.mark.parametrize("kw", [
    dict(random_map_start_position=(1, 1, "west")),                    # not a border tile
    dict(random_map_start_position=(0, 1, "north"), random_map_width=3, random_map_height=3),
    dict(random_map_start_position=(0, -1, "west"), random_map_goal_position=(0, -1, "west")),
    dict(random_map_minimum_distance_between_start_and_goal=2),        # needs 'random'
    dict(random_map_start_position="random", random_map_goal_position="random",
         random_map_minimum_distance_between_start_and_goal=7),        # > w + h - 2
    dict(random_map_start_position="nowhere"),
])
def test_start_goal_validation_raises_value_error(kw):
    with pytest.raises(ValueError):
        C.make_spec(**kw)


def test_unknown_kwarg_is_a_type_error():
    with pytest.raises(TypeError):
        C.make_spec(not_a_kwarg=1)


def test_warnings_like_reference():
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        C.make_spec(traffic_density=0.2, features_to_include_in_observation=["walls"])
    assert any("Traffic is generated" in str(x.message) for x in w)


def test_feature_channels_follow_reference_dict_keys():
    ch = C.feature_channels(["walls", "traffic_light", "sand", "nonexistent", "car_lane all right"])
    keys = [k for k, _ in ch]
    assert keys == ["walls", "traffic_light_green", "traffic_light_yellow", "traffic_light_red", "sand",
                    "nonexistent", "car_lane all right"]
    codes = dict(ch)
    assert codes["nonexistent"] == C.CH_ZERO and codes["car_lane all right"] == C.CH_LANE0 + 31
    # the generic pass overwrites an explicitly listed traffic_light_green (always zero then)
    assert dict(C.feature_channels(["traffic_light", "traffic_light_green"]))["traffic_light_green"] == C.CH_ZERO


@pytest.mark.parametrize("lo,hi", [(0.5, 10.0), (0.0, 0.0), (1.4142135623730951, 3.0), (2.5, 2.2)])
def test_speed_bounds_equal_fp64_norm(lo, hi):
    smin, smax = C._speed_sq_bounds(lo, hi)
    for s in range(0, 2000):
        assert (smin <= s <= smax) == (lo <= math.sqrt(s) <= hi), s


def test_rule_compilation():
    r = C.compile_rule(C.DEFAULT_RULES[1])
    assert r.tile_exits == 0b0111  # "1110" = north, east, south
    sn = C.AGENT_DIRECTIONS.index("south_to_north")
    assert r.weight[sn][C.ROUTES.index("west_to_east")] == 1
    assert sum(map(sum, r.weight)) == 3
    spec = C.make_spec()
    with pytest.raises(ValueError):
        C.add_rule(spec, C.DEFAULT_RULES[0])
    assert C.remove_rule(spec, "t_intersection_brake") and len(spec.rules) == 1


def test_json_map_loader_roundtrip(tmp_path):
    import helpers
    m = C.json_file_to_map_plan(helpers.TESTDATA + "/4x1_map")
    assert (m.width, m.height, m.start, m.goal) == (4, 1, (0, 0, 3), (3, 0, 1))
    assert C.MapPlanArrays.from_dict(m.to_dict()) == m
    old = tmp_path / "old.json"
    old.write_text('{"width": 1, "height": 1, "map": [[{"exits": [0, 1, 0, 1]}]]}')
    with pytest.raises(KeyError):
        C.json_file_to_map_plan(str(old))


def test_feature_vocabulary_and_unknown_names_fit():
    """The whole vocabulary plus unknown names (zero channels) is accepted, as the reference accepts
    any feature list; past PGTG_MAX_CHANNELS distinct keys the build refuses."""
    import pytest
    names = ["walls", "goals", "traffic", "traffic_light"] + list(C._GENERIC) + [f"x{k}" for k in range(14)]
    s = C.make_spec(random_map_width=4, random_map_height=4, features_to_include_in_observation=names)
    assert len(s.channels) == 61
    with pytest.raises(ValueError):
        C.make_spec(features_to_include_in_observation=[f"x{k}" for k in range(C.MAX_CHANNELS + 1)])
