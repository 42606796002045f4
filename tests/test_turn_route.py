"""Turn-aware route choice (DESIGN.md §3 rule 4; SURVEY Appendix B: the
transition route minimises distance plus turn penalty, auto costing's
turn_penalty_factor 200, py/generate_test_trace.py:93-96): a known-answer case
on a hand-built block where the distance-shortest route and the cost-shortest
route differ, so the matched OSMLR segments name the route the rule picked.

    E <----------- D ---- C        vehicle: p0 on A->B heading east, p1 on D->E
                    \\     |        route 1: B->D, 56.6 m, one 135-degree turn
                     \\    |                 (73.6 m) + 45 degrees into D->E (10 m)
    A -------------> B              route 2: B->C->D, 80 m, two 90-degree turns
                                             (2 x 27.1 m) + straight into D->E (3.7 m)

With factor 200 route 2 costs less (137.7 vs 140.2 m); with factor 0 the
distance decides (route 1)."""
import math

import numpy as np
import pytest

import handgraph

LAT = 40.0
MLAT = 20037581.187 / 180.0           # metres per degree of latitude (equirectangular)
MLON = MLAT * math.cos(math.radians(LAT))


def _pt(x, y):
    return (LAT + y / MLAT, x / MLON)


@pytest.fixture(scope="module")
def block(tmp_path_factory):
    d = tmp_path_factory.mktemp("turn")
    nodes = [_pt(-300, 0), _pt(0, 0), _pt(0, 40), _pt(-40, 40), _pt(-300, 40)]  # A B C D E
    segs = [(8, None), (16, None), (24, None), (32, None), (40, None)]
    from handgraph import SEG_BEGIN, SEG_END
    fl = SEG_BEGIN | SEG_END
    edges = [dict(**{"from": 0, "to": 1}, seg=0, flags=fl, level=0),  # A->B
             dict(**{"from": 1, "to": 2}, seg=1, flags=fl, level=0),  # B->C
             dict(**{"from": 2, "to": 3}, seg=2, flags=fl, level=0),  # C->D
             dict(**{"from": 1, "to": 3}, seg=3, flags=fl, level=0),  # B->D
             dict(**{"from": 3, "to": 4}, seg=4, flags=fl, level=0)]  # D->E
    path = str(d / "block.otmg")
    handgraph.write(path, nodes, edges, segs)
    return path


def _batch():
    pts = [_pt(-150, 0), _pt(-60, 0), _pt(-150, 40), _pt(-220, 40)]
    return dict(trace_off=np.array([0, 4], np.int64), lat=np.array([p[0] for p in pts], np.float32),
                lon=np.array([p[1] for p in pts], np.float32), time=np.array([0.0, 6.0, 20.0, 26.0]),
                accuracy=np.full(4, 5.0, np.float32))


MEILI = dict(search_radius=15.0, max_search_radius=15.0, gps_accuracy=5.0)


@pytest.mark.parametrize("factor,want", [(200.0, [8, 16, 24, 40]), (0.0, [8, 32, 40])])
def test_route_choice_known_answer(block, oracle, factor, want):
    r = oracle.match_batch(oracle.Graph(block), _batch(), p=oracle.params(turn_penalty_factor=factor, **MEILI))
    assert list(r["segments"]["segment_id"]) == want


@pytest.mark.gpu
@pytest.mark.parametrize("factor", [200.0, 0.0])
def test_route_choice_gpu(block, oracle, results_equal, factor):
    from reporter_amd import Engine
    with Engine(graph_path=block, turn_penalty_factor=factor, **MEILI) as eng:
        res = eng.match(_batch())
    orc = oracle.match_batch(oracle.Graph(block), _batch(), p=oracle.params(turn_penalty_factor=factor, **MEILI))
    results_equal(orc, res, "turn factor %g" % factor)
