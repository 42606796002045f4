"""Interpolated points (CPU, the oracle): the rule of DESIGN.md §3 rule 7.

SURVEY Appendix B: a point within interpolation_distance of the previous
column gets no HMM state and is "projected onto the final route afterwards".
README.md:162-163 defines a segment's begin/end_shape_index as "the index in
the original trace before/at the start/end of the segment".  These cases pin
the placement, the monotone filter, the shape indices and the boundary times on
a hand-built road where every number can be worked out on paper.
"""
import math

import numpy as np
import pytest

import handgraph

MPD = 20037581.187 / 180.0


@pytest.fixture(scope="module")
def road(tmp_path_factory):
    d = tmp_path_factory.mktemp("hand")
    path, fwd = handgraph.straight_road(str(d / "road.otmg"), lat=40.0, lon0=0.0, step_deg=0.001, n_nodes=5)
    return path, fwd


def _batch(traces, lat=40.0, acc=5.0):
    lon = np.concatenate([np.array([p[0] for p in t], np.float32) for t in traces])
    tm = np.concatenate([np.array([p[1] for p in t], np.float64) for t in traces])
    off = np.zeros(len(traces) + 1, np.int64)
    off[1:] = np.cumsum([len(t) for t in traces])
    return dict(trace_off=off, lat=np.full(len(lon), lat, np.float32), lon=lon, time=tm,
                accuracy=np.full(len(lon), acc, np.float32))


def _x(lon, lat=40.0):
    """metres east of lon 0 along the road (equirectangular, double)"""
    return lon * MPD * math.cos(math.radians(lat))


# p0 state on edge 0 at ~17 m; p1 placed (+4.3 m); p2 behind p1 (unplaced);
# p3 placed (+8.5 m); p4 state on edge 1; p5 state on edge 2
TRACE_A = [(0.0002, 0.0), (0.00025, 1.0), (0.00022, 2.0), (0.0003, 3.0), (0.0011, 10.0), (0.0021, 20.0)]


def test_placement_and_monotone_filter(road, oracle):
    path, _ = road
    r = oracle.match_batch(oracle.Graph(path), _batch([TRACE_A]), keep_stages=True)
    ip = r["ipos"]
    assert ip[0] == -1.0 and ip[4] == -1.0 and ip[5] == -1.0  # states
    # p2 is placed behind p1 (the monotone filter makes it no anchor: the
    # boundaries below never name it)
    assert 0 < ip[2] < ip[1]
    for k in (1, 3):
        assert abs(ip[k] - (_x(TRACE_A[k][0]) - _x(TRACE_A[0][0]))) < 1e-3
    assert ip[1] < ip[3]


def test_shape_indices_before_at_boundary(road, oracle):
    path, _ = road
    r = oracle.match_batch(oracle.Graph(path), _batch([TRACE_A]), keep_stages=True)
    s = r["segments"]
    assert list(s["segment_id"]) == [8, 16, 24]
    # the node between edge 0 and edge 1 (x ~ 85.3 m) lies past p3 (~25.6 m):
    # the last point at or before it is p3 (index 3), not the state p0
    assert list(s["begin_shape_index"]) == [0, 3, 4]
    assert list(s["end_shape_index"]) == [3, 4, 5]
    # boundary time between the anchors around it (p3 at t=3 and p4 at t=10)
    x0, x3, x4 = (_x(TRACE_A[k][0]) for k in (0, 3, 4))
    node1 = _x(0.001)
    t_node1 = 3.0 + 7.0 * ((node1 - x3) / (x4 - x3))
    assert s["end_time"][0] == pytest.approx(t_node1, rel=1e-6)
    assert s["start_time"][1] == s["end_time"][0]
    # without placed points the rule is the two-state one: node 2 between p4 and p5
    x5 = _x(TRACE_A[5][0])
    t_node2 = 10.0 + 10.0 * ((_x(0.002) - x4) / (x5 - x4))
    assert s["end_time"][1] == pytest.approx(t_node2, rel=1e-6)


def test_points_after_last_state_are_unplaced(road, oracle):
    # interpolated points after the chain's last state have no step route
    path, _ = road
    tr = [(0.0002, 0.0), (0.0012, 10.0), (0.00122, 11.0), (0.00125, 12.0)]
    r = oracle.match_batch(oracle.Graph(path), _batch([tr]), keep_stages=True)
    assert list(r["ipos"][2:]) == [-1.0, -1.0]
    s = r["segments"]
    # the chain ends at the state p1 (index 1); the points after it count nowhere
    assert list(s["end_shape_index"]) == [0, 1]


def test_stationary_stop_is_placed_at_its_state(road, oracle):
    # a vehicle standing at p0 (exact repeats) then driving on: the repeats sit
    # at position 0, so the boundary's "before/at" index is the last of them
    path, _ = road
    tr = [(0.0005, 0.0), (0.0005, 5.0), (0.0005, 10.0), (0.0005, 15.0), (0.0015, 25.0)]
    r = oracle.match_batch(oracle.Graph(path), _batch([tr]), keep_stages=True)
    assert list(r["ipos"]) == [-1.0, 0.0, 0.0, 0.0, -1.0]
    s = r["segments"]
    assert list(s["segment_id"]) == [8, 16]
    assert list(s["end_shape_index"]) == [3, 4]
    # the node is reached after the stop: time linear from p3 (t=15) to p4
    x0, x4 = _x(0.0005), _x(0.0015)
    t = 15.0 + 10.0 * ((_x(0.001) - x0) / (x4 - x0))
    assert s["end_time"][0] == pytest.approx(t, rel=1e-6)


def test_two_state_rule_unchanged_without_interpolated_points(road, oracle):
    path, _ = road
    tr = [(0.0002, 0.0), (0.0011, 10.0), (0.0021, 20.0)]
    r = oracle.match_batch(oracle.Graph(path), _batch([tr]), keep_stages=True)
    s = r["segments"]
    assert list(s["begin_shape_index"]) == [0, 0, 1]
    assert list(s["end_shape_index"]) == [0, 1, 2]
    x0, x1 = _x(0.0002), _x(0.0011)
    assert s["end_time"][0] == pytest.approx(10.0 * (_x(0.001) - x0) / (x1 - x0), rel=1e-6)


def test_shape_used_can_land_on_an_interpolated_point(road, oracle):
    # shape_used = begin_shape_index of the trim segment (py/reporter_service.py:116-127)
    path, _ = road
    tr = [(0.0002, 0.0), (0.00028, 1.0), (0.0012, 30.0), (0.0022, 40.0), (0.0032, 50.0)]
    r = oracle.match_batch(oracle.Graph(path), _batch([tr]), keep_stages=True)
    assert r["ipos"][1] > 0
    s = r["segments"]
    assert list(s["begin_shape_index"])[:2] == [0, 1]
    assert r["traces"]["shape_used"][0] == 1


# DESIGN.md §3 rule 4: a probe that projects behind the previous column on the
# same directed edge is a stay (GPS noise; vehicles do not reverse): route
# distance 0, no traversal, no U-turn onto the opposite edge and back.
# x: 17 m, 51 m, 38 m (13 m behind: a column, not interpolated), 77 m, then edge 2.
TRACE_BACK = [(0.0002, 0.0), (0.0006, 5.0), (0.00045, 10.0), (0.0009, 15.0), (0.0014, 20.0)]


def test_backward_probe_on_same_edge_is_a_stay(road, oracle):
    path, fwd = road
    r = oracle.match_batch(oracle.Graph(path), _batch([TRACE_BACK]), keep_stages=True)
    e = [int(r["cand_edge"][i * 32 + s]) for i, s in enumerate(r["state"])]
    o = [float(r["cand_off"][i * 32 + s]) for i, s in enumerate(r["state"])]
    assert e[:4] == [fwd[0]] * 4 and e[4] == fwd[1]
    assert o[2] < o[1]  # behind the previous column
    assert r["route_dist"][2] == 0.0
    # the next step starts from the stay's own offset (the HMM's state)
    assert r["route_dist"][3] == pytest.approx(o[3] - o[2], abs=1e-4)
    s = r["segments"]
    assert list(s["segment_id"]) == [8, 16]  # no opposite-direction segment
    assert list(s["begin_shape_index"]) == [0, 3] and list(s["end_shape_index"]) == [3, 4]
    t = 15.0 + 5.0 * ((_x(0.001) - _x(0.0009)) / (_x(0.0014) - _x(0.0009)))
    assert s["end_time"][0] == pytest.approx(t, rel=1e-6)


def test_chain_ending_on_a_stay_ends_at_the_farthest_offset(road, oracle):
    # the last state is the stay: the traversal still ends at 51 m (the
    # farthest offset reached), timed and indexed at the last state
    path, _ = road
    r = oracle.match_batch(oracle.Graph(path), _batch([TRACE_BACK[:3]]), keep_stages=True)
    s = r["segments"]
    assert list(s["segment_id"]) == [8]
    assert list(s["begin_shape_index"]) == [0] and list(s["end_shape_index"]) == [2]
    assert s["length"][0] == -1
