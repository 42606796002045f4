"""No spec limits (VERDICT r3 "next" #6): a probe with more than 256 distinct
edges within its radius, and a route search past 98,304 labels, are matched
like any other -- no 500, GPU and oracle bit-identical.

Until round 3 both cases failed the trace ("too many candidate edges within
search radius" / "route search exceeded node limit"), a limit of this
implementation the reference does not have.  Now the oracle grows its
workspace, and the GPU path hands such probes / searches to tiers whose HBM
tables the host sizes on demand (kernels.h CAND_BIG_SLOTS, HUGE_SLOTS; the
batch is redone after a grow).

  star: 200 two-way spokes of 90 m around one hub (handgraph.star): every
        probe within 100 m of the hub sees 400 directed edges.
  grid: a 12 x 12 km synthetic city with 32 m blocks (~640k directed
        edges), probes 600 s apart (gaps of 0.5-2.2 km), no turn penalty: the
        search bound (5 x the gap) reaches much of the graph, ~145k edge
        labels per search.
"""
import math

import numpy as np
import pytest

from reporter_amd import encode_request, synth

import handgraph

KMAX = 32
SPOKES = 200
STAR_LON = 10.0
RADIUS_100 = dict(search_radius=100.0, max_search_radius=100.0)
# no turn penalty and a 4 km breakage: searches reach across most of the grid
GRID_MEILI = dict(search_radius=15.0, max_search_radius=15.0, turn_penalty_factor=0.0, breakage_distance=4000.0)


@pytest.fixture(scope="module")
def star(tmp_path_factory):
    # lon 10: the request encoder (DecimalFormat("###.######"), Point.java:29)
    # writes |x| < 1 as ".5", which the server's JSON parser rejects
    path, out, inn = handgraph.star(str(tmp_path_factory.mktemp("star") / "star.otmg"), lon=STAR_LON,
                                    n_spokes=SPOKES, length_m=90.0)
    return path, out, inn


@pytest.fixture(scope="module")
def dense_grid(tmp_path_factory):
    d = tmp_path_factory.mktemp("dense")
    return synth.make_graph(str(d / "grid32.otmg"), width_m=12000, height_m=12000, block_m=32, jitter_m=0,
                            arterial_every=8, highway_every=1000, complex_every=4, seg_max_m=300)


def _star_point(i, d, lat=40.0, lon=STAR_LON):
    a = 2.0 * math.pi * i / SPOKES
    return lat + d * math.cos(a) / handgraph.MPD, lon + d * math.sin(a) / (handgraph.MPD * math.cos(math.radians(lat)))


def star_batch():
    """Three traces through the hub: in on spoke 0 and out on 100; in on 37
    and out on 60 (a 41 degree turn); a probe on the hub itself."""
    traces = [
        [(0, 80), (0, 45), (0, 12), (100, 15), (100, 50), (100, 85)],
        [(37, 85), (37, 30), (37, 3), (60, 25), (60, 60)],
        [(10, 60), (10, 0.5), (150, 70)],
    ]
    lat, lon, off = [], [], [0]
    for tr in traces:
        for i, d in tr:
            la, lo = _star_point(i, d)
            lat.append(la)
            lon.append(lo)
        off.append(len(lat))
    n = len(lat)
    tm = np.concatenate([np.arange(len(tr)) * 6.0 + 1000.0 * k for k, tr in enumerate(traces)])
    return dict(trace_off=np.array(off, np.int64), lat=np.array(lat, np.float32), lon=np.array(lon, np.float32),
                time=tm.astype(np.float64), accuracy=np.full(n, 5.0, np.float32))


def grid_batch(graph):
    return synth.make_traces(graph, 3, 6, interval_s=600.0, noise_sigma_m=5.0, accuracy=5.0, seed=5)


def _edges_within(graph, lat, lon, r):
    """Directed edges with an end node within r metres (a lower bound of the
    edges whose projection is within r)."""
    nla = synth._graph_section(graph, 0, np.float32).astype(np.float64)
    nlo = synth._graph_section(graph, 1, np.float32).astype(np.float64)
    ef = synth._graph_section(graph, 3, np.int32)
    et = synth._graph_section(graph, 4, np.int32)
    mpd = handgraph.MPD
    dy = (nla - lat) * mpd
    dx = (nlo - lon) * mpd * math.cos(math.radians(lat))
    near = np.hypot(dx, dy) <= r
    return int(np.count_nonzero(near[ef] | near[et]))


def _bodies(b):
    out = []
    for t in range(len(b["trace_off"]) - 1):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        out.append(encode_request("veh%d" % t, b["lat"][a:e], b["lon"][a:e], b["time"][a:e].astype(np.int64),
                                  b["accuracy"][a:e].astype(np.int32)))
    return out


# ---------------------------------------------------------------- oracle (CPU)

def test_star_has_more_edges_than_the_old_limit(star):
    path, _, _ = star
    b = star_batch()
    for la, lo in zip(b["lat"], b["lon"]):
        assert _edges_within(path, float(la), float(lo), 100.0) > 256


def test_oracle_star_matches(star, oracle):
    path, out, inn = star
    b = star_batch()
    r = oracle.match_batch(oracle.Graph(path), b, p=oracle.params(**RADIUS_100), keep_stages=True)
    assert (r["traces"]["error_kind"] == 0).all()
    assert (r["ncand"] == KMAX).all()
    e = [int(r["cand_edge"][i * KMAX + s]) for i, s in enumerate(r["state"])]
    assert e[:6] == [inn[0]] * 3 + [out[100]] * 3
    # at 1.8 degrees between spokes the emission costs of neighbouring spokes
    # differ by hundredths: the transitions pick among them
    assert all(any(x == inn[k] for k in range(34, 41)) for x in e[6:9])
    assert all(any(x == out[k] for k in range(57, 64)) for x in e[9:11])
    seg = r["segments"]["segment_id"]
    assert 101 << 3 in seg and len(seg) >= 5
    for body in _bodies(b):
        code, resp = oracle.handle_request(oracle.Graph(path), body, p=oracle.params(**RADIUS_100))
        assert code == 200, resp[:200]


def test_oracle_long_gaps_on_dense_grid(dense_grid, oracle):
    b = grid_batch(dense_grid)
    r = oracle.match_batch(oracle.Graph(dense_grid), b, p=oracle.params(**GRID_MEILI), keep_stages=True, nthreads=3)
    assert (r["traces"]["error_kind"] == 0).all()
    # searches bounded by 5 x gaps of 0.5-2.2 km on a 32 m grid: their edge
    # departure labels alone (the oracle's nodes_settled) past the old
    # 98,304-label limit on average
    c = r["counters"]
    assert c["searches"] >= 6 and c["route_searches"] >= 6
    assert c["nodes_settled"] / c["searches"] > 98304
    assert c["route_nodes_settled"] / c["route_searches"] > 98304
    assert (r["state"] >= 0).sum() >= len(b["lat"]) // 2
    for body in _bodies(b):
        code, resp = oracle.handle_request(oracle.Graph(dense_grid), body, p=oracle.params(**GRID_MEILI))
        assert code == 200, resp[:200]


# ---------------------------------------------------------------- GPU parity

def _gpu_vs_oracle(graph, b, meili, oracle, results_equal):
    from reporter_amd import Engine
    from test_gpu_parity import _stage_compare
    orc = oracle.match_batch(oracle.Graph(graph), b, p=oracle.params(**meili), keep_stages=True, nthreads=3)
    with Engine(graph_path=graph, **meili) as eng:
        res = eng.match(b)
        first = eng.spill_stats()
        _stage_compare(eng, orc, b)
        results_equal(orc, res, "final")
        res2 = eng.match(b)  # the tables are sized now: one run, same results
        second = eng.spill_stats()
        results_equal(orc, res2, "repeat")
        got = eng.report_batch(_bodies(b))
    g = oracle.Graph(graph)
    for body, (code, resp) in zip(_bodies(b), got):
        assert code == 200, resp[:200]
        assert (code, resp) == oracle.handle_request(g, body, p=oracle.params(**meili))
    return first, second


@pytest.mark.gpu
@pytest.mark.parametrize("path_kind", ["large", "small"])
def test_gpu_star_candidate_hbm_tier(star, oracle, results_equal, monkeypatch, path_kind):
    monkeypatch.setenv("OTM_SMALL_POINTS", "0" if path_kind == "large" else str(1 << 40))
    path, _, _ = star
    first, second = _gpu_vs_oracle(path, star_batch(), RADIUS_100, oracle, results_equal)
    assert first["cand_big"] == len(star_batch()["lat"])  # every probe: 400 edges
    assert first["attempts"] >= 2  # the tables were made on demand ...
    assert second["attempts"] == 1 and second["cand_big"] == first["cand_big"]  # ... and kept
    # the runs for the tier's growth resumed at the candidate HBM tier (round
    # 6); a transition-matrix overflow in the same batch still redoes it whole
    assert first["resumed"] >= 1 and second["resumed"] == 0
    assert second["cand_wave"] == first["cand_wave"]  # the spill snapshots survive the resume


@pytest.mark.gpu
def test_gpu_long_gaps_huge_search_tier(dense_grid, oracle, results_equal):
    first, second = _gpu_vs_oracle(dense_grid, grid_batch(dense_grid), GRID_MEILI, oracle, results_equal)
    assert first["trans_huge"] > 0 and first["route_huge"] > 0
    assert first["attempts"] >= 2
    assert second["attempts"] == 1
    # the runs after the first resumed at the huge tier of the transition or
    # route stage (round 6); the spill snapshots equal the clean run's
    assert first["resumed"] >= 1 and second["resumed"] == 0
    for k in ("cand_wave", "trans_online", "trans_global", "route_online", "route_global", "trans_huge",
              "route_huge"):
        assert first[k] == second[k], k


@pytest.mark.gpu
@pytest.mark.parametrize("why", ["cap", "oom"])
@pytest.mark.parametrize("tier", ["cand", "huge"])
def test_gpu_tables_that_cannot_grow_fail_their_traces_only(star, dense_grid, oracle, results_equal, monkeypatch,
                                                           tier, why):
    """Past the on-demand tiers' growth cap (kernels.h HUGE_MAX_LOG2 /
    CAND_MAX_LOG2, lowered to 0 here: no tables at all) or out of HBM, a probe
    or search that needs the tier fails its own trace with the 500 the
    reference sends for a matcher exception (error_kind CAND_OVERFLOW /
    SEARCH_OVERFLOW); every other trace of the batch matches the oracle
    (round 4 failed the whole batch).  why="oom": the growth's
    hipMalloc really fails (OTM_TEST_GROW_OOM asks for 2^62 bytes): the same
    traces-only 500s, the runtime's error cleared, and for that batch only --
    the next batch on the same engine grows the tier and matches every trace
    (ADVICE r5)."""
    from reporter_amd import Engine
    if why == "oom":
        monkeypatch.setenv("OTM_TEST_GROW_OOM", "1")
    if tier == "cand":
        if why == "cap":
            monkeypatch.setenv("OTM_CAND_MAX_LOG2", "0")
        graph, meili = star[0], dict(search_radius=20.0, max_search_radius=20.0)
        b = star_batch()  # traces 0-2 each hold a probe within 20 m of the hub (400 edges)
        lat, lon = zip(*[_star_point(5, 85), _star_point(5, 60), _star_point(6, 40)])  # + one that never nears it
        b = dict(trace_off=np.append(b["trace_off"], len(b["lat"]) + 3),
                 lat=np.append(b["lat"], np.array(lat, np.float32)), lon=np.append(b["lon"], np.array(lon, np.float32)),
                 time=np.append(b["time"], 5000.0 + np.arange(3) * 6.0),
                 accuracy=np.append(b["accuracy"], np.full(3, 5.0, np.float32)))
        kind, failing = 2, [0, 1, 2]
    else:
        if why == "cap":
            monkeypatch.setenv("OTM_HUGE_MAX_LOG2", "0")
        graph, meili = dense_grid, GRID_MEILI
        far = grid_batch(dense_grid)  # 600 s gaps: searches past the global tier
        near = synth.make_traces(dense_grid, 2, 6, interval_s=5.0, noise_sigma_m=5.0, accuracy=5.0, seed=6)
        b = {k: np.concatenate([far[k], near[k]]) for k in ("lat", "lon", "time", "accuracy")}
        b["trace_off"] = np.concatenate([far["trace_off"], far["trace_off"][-1] + near["trace_off"][1:]])
        kind, failing = 3, None
    with Engine(graph_path=graph, **meili) as eng:
        res = eng.match(b)
        sp = eng.spill_stats()
        again = None
        if why == "oom":
            monkeypatch.delenv("OTM_TEST_GROW_OOM")
            again = eng.match(b)
    orc = oracle.match_batch(oracle.Graph(graph), b, p=oracle.params(**meili), nthreads=4)
    if again is not None:
        results_equal(orc, again, "after the out-of-HBM batch")
    tr = res.traces
    bad = [t for t in range(len(tr)) if tr["code"][t] != 200]
    if failing is not None:
        assert bad == failing
    else:
        assert bad and len(bad) < len(tr) and sp["trans_huge"] + sp["route_huge"] > 0
    for t in bad:
        assert tr["code"][t] == 500 and tr["error_kind"][t] == kind
    ok = [t for t in range(len(tr)) if t not in bad]
    assert all(orc["traces"]["code"][t] == 200 for t in range(len(tr)))
    for t in ok:  # every other trace: the oracle's records (way ids by their own offsets)
        a, n = tr["seg_off"][t], tr["seg_cnt"][t]
        oa, on = orc["traces"]["seg_off"][t], orc["traces"]["seg_cnt"][t]
        assert n == on
        gs, os_ = res.segments[a:a + n], orc["segments"][oa:oa + on]
        for f in gs.dtype.names:
            if f != "way_off":
                assert np.array_equal(gs[f], os_[f]), f
        for x, y in zip(gs, os_):
            assert np.array_equal(res.way_ids[x["way_off"]:x["way_off"] + x["way_cnt"]],
                                  orc["way_ids"][y["way_off"]:y["way_off"] + y["way_cnt"]])
        ra, rn = tr["rep_off"][t], tr["rep_cnt"][t]
        ora, orn = orc["traces"]["rep_off"][t], orc["traces"]["rep_cnt"][t]
        assert res.reports[ra:ra + rn].tobytes() == orc["reports"][ora:ora + orn].tobytes()


@pytest.mark.gpu
def test_gpu_resume_equals_whole_redo(dense_grid, oracle, results_equal, monkeypatch):
    """A batch of ordinary traces with one whose 600 s gaps need the huge
    search tier: on a fresh engine the tier's tables are made on demand and
    the batch resumes at that tier (round 6) -- its results equal a whole
    redo's (OTM_NO_RESUME, rounds 1-5), a clean run's on tables already
    grown, and the oracle's."""
    from reporter_amd import Engine
    normal = synth.make_traces(dense_grid, 300, 30, interval_s=5.0, noise_sigma_m=5.0, accuracy=5.0, seed=11)
    far = grid_batch(dense_grid)
    b = {k: np.concatenate([normal[k], far[k]]) for k in ("lat", "lon", "time", "accuracy")}
    b["trace_off"] = np.concatenate([normal["trace_off"], normal["trace_off"][-1] + far["trace_off"][1:]])
    with Engine(graph_path=dense_grid, **GRID_MEILI) as eng:
        first = eng.match(b)
        st1 = eng.spill_stats()
        clean = eng.match(b)
        st2 = eng.spill_stats()
    monkeypatch.setenv("OTM_NO_RESUME", "1")
    with Engine(graph_path=dense_grid, **GRID_MEILI) as eng:
        whole = eng.match(b)
        st3 = eng.spill_stats()
    assert st1["attempts"] >= 2 and st1["resumed"] >= 1
    assert st2["attempts"] == 1 and st3["resumed"] == 0 and st3["attempts"] >= 2
    orc = oracle.match_batch(oracle.Graph(dense_grid), b, p=oracle.params(**GRID_MEILI), nthreads=4)
    results_equal(orc, first, "resumed")
    results_equal(orc, clean, "clean")
    results_equal(orc, whole, "whole redo")
