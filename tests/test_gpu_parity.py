"""GPU parity: libotmatch's HIP path vs the CPU oracle, bit for bit.

Every comparison goes through the C ABI (reporter_amd.Engine ->
libotmatch.so).  Integer / index outputs and the float stage outputs are
compared exactly: the kernels follow the oracle's float evaluation order with
FMA contraction off.  Times and speeds are doubles computed by
the same expressions, also compared exactly (north star allows 1e-3
relative; we hold ourselves to 0).
"""
import json

import numpy as np
import numpy.testing as npt
import pytest

from reporter_amd import Engine, encode_request, synth

pytestmark = pytest.mark.gpu

KMAX = 32


@pytest.fixture(params=["large", "small"])
def batch_path(request, monkeypatch):
    """The two launch plans of a batch: "large" = spatial work
    order + lane-tier candidates, "small" (under OTM_SMALL_POINTS points,
    the batcher's rounds) = natural order, one wave per probe.  The tests'
    batches are small, so the threshold is forced either way."""
    monkeypatch.setenv("OTM_SMALL_POINTS", "0" if request.param == "large" else str(1 << 40))
    return request.param


def _stage_compare(eng, orc, batch):
    P = len(batch["lat"])
    nc_g = eng.debug("ncand")[:P]
    npt.assert_array_equal(nc_g, orc["ncand"], err_msg="ncand")
    mask = (np.arange(KMAX)[None, :] < nc_g[:, None]).ravel()
    for name in ("cand_edge", "cand_off", "cand_emis"):
        g = eng.debug(name)[:P * KMAX]
        npt.assert_array_equal(g[mask], orc[name][mask], err_msg=name)
    npt.assert_array_equal(eng.debug("gc")[:P], orc["gc"], err_msg="gc")
    npt.assert_array_equal(eng.debug("col_prev")[:P], orc["col_prev"], err_msg="col_prev")
    toff = eng.debug("trans_off")[:P + 1]
    npt.assert_array_equal(toff, orc["trans_off"], err_msg="trans_off")
    # transitions of traces without errors (the oracle skips errored traces)
    ok_pts = np.zeros(P, bool)
    tr = orc["traces"]
    off = batch["trace_off"]
    for t in range(len(tr)):
        if tr["error_kind"][t] == 0:
            ok_pts[off[t]:off[t + 1]] = True
    tg = eng.debug("trans")
    sel = np.zeros(int(toff[-1]), bool)
    for p in np.nonzero(ok_pts & (orc["col_prev"] >= 0))[0]:
        sel[toff[p]:toff[p + 1]] = True
    npt.assert_array_equal(tg[:len(sel)][sel], orc["trans"][sel], err_msg="trans")
    npt.assert_array_equal(eng.debug("state")[:P], orc["state"], err_msg="state")
    npt.assert_array_equal(eng.debug("route_dist")[:P], orc["route_dist"], err_msg="route_dist")
    # interpolated points' positions on their step's route (K7a)
    npt.assert_array_equal(eng.debug("ipos")[:P][ok_pts], orc["ipos"][ok_pts], err_msg="ipos")


def _run_both(graph, batch, oracle, results_equal, meili=None, stages=True, counters=True, index_radius_m=None,
              grid_mult=None, trans_lanes=None, index_near_m=None):
    meili = meili or {}
    with Engine(graph_path=graph, index_radius_m=index_radius_m, grid_mult=grid_mult, trans_lanes=trans_lanes,
                index_near_m=index_near_m, **meili) as eng:
        eng.set_counting(counters)
        res = eng.match(batch)
        p = oracle.params(**meili)
        orc = oracle.match_batch(oracle.Graph(graph), batch, p=p, keep_stages=True, nthreads=4)
        if stages:
            _stage_compare(eng, orc, batch)
        results_equal(orc, res, "final")
        if counters:
            c = eng.counters()
            # the cells / entries a probe visits depend on the device grid's
            # cell size (otm_grid_info): equal to the oracle's on the file grid
            grid_keys = ("cells_visited", "cell_entries_scanned")
            same_grid = eng.grid_info()["mult"] == 1
            for k, v in orc["counters"].items():
                if (k in grid_keys and not same_grid) or k not in c:  # (oracle-only: §8(d)'s unique-edge term)
                    continue
                assert c[k] == v, "counter %s gpu %d oracle %d" % (k, c[k], v)
        return res, orc


@pytest.mark.parametrize("radius", [None, 0.0, 300.0], ids=["index_default", "no_index", "index300"])
@pytest.mark.parametrize("grid_mult", [None, 1, 3], ids=["grid_auto", "grid1", "grid3"])
def test_city_sample_sigma15(small_graph, oracle, results_equal, batch_path, radius, grid_mult):
    # the distance index answers columns whose bound fits its radius; the rest
    # (and everything when it is disabled) run the online search tiers; the
    # device grid's cells are the file's, merged 3 x 3, or the auto choice --
    # results must be identical in every configuration
    b = synth.make_traces(small_graph, 200, 100, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=11)
    res, orc = _run_both(small_graph, b, oracle, results_equal, index_radius_m=radius, grid_mult=grid_mult)
    assert (res.traces["code"] == 200).mean() > 0.95
    assert len(res.segments) > 1000 and len(res.reports) > 50


@pytest.mark.parametrize("near", [[], [300.0], [150.0, 300.0, 600.0]], ids=["none", "one", "three"])
def test_near_indexes(small_graph, oracle, results_equal, near):
    # columns probe the smallest near index covering their bound (the same
    # rows at a smaller radius), the rest the full index: every stage, route
    # and counter identical to the oracle with none, one or three levels.
    # 15 s sampling spreads the bounds (5 x gc) over all of them.
    b = synth.make_traces(small_graph, 200, 60, interval_s=15.0, noise_sigma_m=15.0, accuracy=15.0, seed=41)
    _run_both(small_graph, b, oracle, results_equal, index_radius_m=1250.0, index_near_m=near)


@pytest.mark.parametrize("lanes", [8, 16])
def test_transition_lanes(small_graph, oracle, results_equal, lanes):
    # k_trans_sub at 8 lanes per column runs two passes (columns of more than
    # OTM_TRANS_KC8 candidates a side go to a 16-lane pass over a device list);
    # 16 lanes run one.  Node candidates merge edges, so K varies per column
    # and both passes see work here.
    b = synth.make_traces(small_graph, 200, 100, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=23)
    res, orc = _run_both(small_graph, b, oracle, results_equal, trans_lanes=lanes)
    k = orc["ncand"]
    assert k.max() > 8 and (k > 0).mean() > 0.9


@pytest.mark.parametrize("grid_mult", [1, None], ids=["grid1", "grid_auto"])
def test_candidate_tiers(small_graph, rural_graph, oracle, results_equal, grid_mult):
    # K2's lane tier (1 lane per probe); probes beyond its edge cap go to the
    # wave tier -- candidates, counters and everything after identical to the
    # oracle.  The rural graph at 100 m has many edges per probe.
    b = synth.make_traces(small_graph, 150, 100, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=31)
    _run_both(small_graph, b, oracle, results_equal, grid_mult=grid_mult)
    b = synth.make_traces(rural_graph, 100, 60, interval_s=30.0, noise_sigma_m=50.0, accuracy=50.0, seed=37)
    _run_both(rural_graph, b, oracle, results_equal, meili={"search_radius": 100.0, "max_search_radius": 100.0},
              grid_mult=grid_mult)


def test_node_candidates(small_graph, oracle, results_equal):
    # SURVEY Appendix B's node snap: end-of-edge projections merge into one
    # candidate per node, carried at offset 0 on the node's first outgoing
    # edge; routes start there with no turn on its side, and a chain never
    # emits a traversal for the edge that only carries a node candidate
    b = synth.make_traces(small_graph, 100, 100, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=29)
    res, orc = _run_both(small_graph, b, oracle, results_equal)
    P = len(b["lat"])
    k = orc["ncand"]
    off = orc["cand_off"].reshape(P, -1)
    edge = orc["cand_edge"].reshape(P, -1)
    node = np.zeros(off.shape, bool)
    for p in range(P):
        node[p, :k[p]] = off[p, :k[p]] == 0.0
        nodes = edge[p, :k[p]][node[p, :k[p]]]
        assert len(np.unique(nodes)) == len(nodes)  # one candidate per node
    assert node.sum() > 0.05 * k.sum()
    st = orc["state"]
    m = st >= 0
    assert (off[np.nonzero(m)[0], st[m]] == 0.0).mean() > 0.02  # matched node states occur


def _auto_index_radius(graph_path, factor=5.0, breakage=2000.0):
    """engine.cpp:auto_index_radius restated: ~140 nodes per row at the
    graph's mean node density, capped at factor x breakage, in 50 m steps."""
    import math
    import struct
    with open(graph_path, "rb") as f:
        hd = f.read(256)
    n = struct.unpack_from("<i", hd, 16)[0]
    bb = struct.unpack_from("<4d", hd, 72)  # min_lat, min_lon, max_lat, max_lon
    lat_mid = 0.5 * (bb[0] + bb[2]) * math.pi / 180.0
    area = max((bb[2] - bb[0]) * 111195.0 * (bb[3] - bb[1]) * 111195.0 * math.cos(lat_mid), 1.0)
    r = min(math.sqrt(140.0 / (2.0 * max(n, 1) / area)), factor * breakage)
    return math.ceil(r / 50.0) * 50.0


def test_index_info(small_graph):
    with Engine(graph_path=small_graph) as eng:
        info = eng.index_info()
        n = eng.graph_info()["nodes"]
        assert info["radius_m"] == pytest.approx(_auto_index_radius(small_graph), abs=50.0)
        assert info["incomplete_rows"] == 0
        assert info["entries"] > 10 * n
    with Engine(graph_path=small_graph, index_radius_m=1250.0) as eng:
        assert eng.index_info()["radius_m"] == 1250.0
    with Engine(graph_path=small_graph, index_radius_m=0) as eng:
        assert eng.index_info()["entries"] == 0
        assert eng.index_levels() == []
    # near indexes: none by default on a small index, else the radii asked
    # below the index's, smallest first, each with fewer entries
    with Engine(graph_path=small_graph, index_radius_m=1250.0) as eng:
        assert eng.index_levels() == []
    with Engine(graph_path=small_graph, index_radius_m=1250.0, index_near_m=[600.0, 300.0, 2000.0]) as eng:
        lv = eng.index_levels()
        assert [x["radius_m"] for x in lv] == [300.0, 600.0]
        assert 0 < lv[0]["entries"] < lv[1]["entries"] < eng.index_info()["entries"]


@pytest.mark.parametrize("expect", ["shrunk", "off"])
def test_index_hbm_budget(small_graph, oracle, results_equal, batch_path, monkeypatch, expect):
    """An index whose slot tables exceed the HBM budget is rebuilt at a
    smaller radius, or left off; results stay identical to the oracle."""
    with Engine(graph_path=small_graph) as eng:
        full = eng.index_info()
    # about a quarter of the full index's slot tables (~40 B per entry: 16-B
    # slots at the default 40 % load): the radius about halves
    budget_mb = str(max(1, full["entries"] * 40 >> 22)) if expect == "shrunk" else "0"
    monkeypatch.setenv("OTM_INDEX_BUDGET_MB", budget_mb)
    with Engine(graph_path=small_graph) as eng:
        info = eng.index_info()
    if expect == "shrunk":
        assert 100.0 <= info["radius_m"] < full["radius_m"]
        assert 0 < info["entries"] < full["entries"]
    else:
        assert info["radius_m"] == 0.0 and info["entries"] == 0
    b = synth.make_traces(small_graph, 200, 60, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=11)
    _run_both(small_graph, b, oracle, results_equal, stages=False, counters=False)


def test_noise_free_traces(small_graph, oracle, results_equal, batch_path):
    b = synth.make_traces(small_graph, 100, 60, interval_s=5.0, noise_sigma_m=0.0, accuracy=0.0, seed=3)
    _run_both(small_graph, b, oracle, results_equal)


@pytest.mark.parametrize("grid_mult", [None, 1, 6], ids=["grid_auto", "grid1", "grid6"])
def test_high_noise_sparse_rural(rural_graph, oracle, results_equal, batch_path, grid_mult):
    b = synth.make_traces(rural_graph, 100, 100, interval_s=30.0, noise_sigma_m=50.0, accuracy=50.0, seed=5)
    with Engine(graph_path=rural_graph, grid_mult=grid_mult, search_radius=100.0) as eng:
        info = eng.grid_info()
    # the sparse state-style graph gets coarse cells when the engine chooses
    assert info["mult"] == grid_mult if grid_mult else info["mult"] >= 3
    _run_both(rural_graph, b, oracle, results_equal, meili=dict(search_radius=100.0, max_search_radius=100.0),
              grid_mult=grid_mult)


def test_long_gaps_force_global_tier(small_graph, oracle, results_equal, batch_path):
    # 120 s sampling: bounds of 5 x gc reach kilometres -> searches overflow
    # the LDS tier and finish in the global-memory tier, same fixed point
    b = synth.make_traces(small_graph, 60, 30, interval_s=120.0, noise_sigma_m=10.0, accuracy=10.0, seed=9)
    _run_both(small_graph, b, oracle, results_equal)


def test_long_traces_mixed_lengths(small_graph, oracle, results_equal, batch_path):
    # traces longer than the Viterbi LDS window (128 points) take the
    # global-memory form, and the segment walk's large LDS plan (129-256
    # points) or its serial walk (longer); mixed with short ones in one batch
    long_b = synth.make_traces(small_graph, 12, 400, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=31)
    mid_b = synth.make_traces(small_graph, 10, 200, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=34)
    short_b = synth.make_traces(small_graph, 40, 30, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=32)
    parts = [long_b, mid_b, short_b]
    offs, base = [np.zeros(1, np.int64)], 0
    for pb in parts:
        offs.append(pb["trace_off"][1:] + base)
        base += pb["trace_off"][-1]
    b = {k: np.concatenate([pb[k] for pb in parts]) for k in ("lat", "lon", "time", "accuracy")}
    b["trace_off"] = np.concatenate(offs)
    _run_both(small_graph, b, oracle, results_equal)


def test_dense_candidates_spill_tiers(small_graph, oracle, results_equal, batch_path):
    # a 300 m search radius puts dozens of distinct edges in range: probes
    # spill from the lane candidate tier to the wave tier, and the candidate
    # count per trace outgrows the Viterbi LDS window
    b = synth.make_traces(small_graph, 30, 60, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=33)
    _run_both(small_graph, b, oracle, results_equal,
              meili=dict(search_radius=300.0, max_search_radius=300.0, max_candidates=32))


def test_edge_cases(small_graph, oracle, results_equal, batch_path):
    base = synth.make_traces(small_graph, 8, 20, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=21)
    lat, lon, tm, acc = (list(base[k]) for k in ("lat", "lon", "time", "accuracy"))
    off = list(base["trace_off"])
    # one-point trace, stationary duplicate points, far-off-graph points, a big gap
    extra = [
        ([lat[0]], [lon[0]], [tm[0]], [15.0]),
        ([lat[1]] * 5, [lon[1]] * 5, [tm[1] + k for k in range(5)], [15.0] * 5),
        ([lat[2] + 1.0, lat[2] + 1.0001], [lon[2], lon[2]], [tm[2], tm[2] + 5], [15.0, 15.0]),
        ([lat[3], lat[60], lat[61]], [lon[3], lon[60], lon[61]], [tm[3], tm[3] + 10, tm[3] + 15], [0.0, -1.0, 500.0]),
    ]
    for la, lo, t, a in extra:
        lat += la
        lon += lo
        tm += t
        acc += a
        off.append(off[-1] + len(la))
    b = dict(trace_off=np.array(off, np.int64), lat=np.array(lat, np.float32), lon=np.array(lon, np.float32),
             time=np.array(tm, np.float64), accuracy=np.array(acc, np.float32))
    _run_both(small_graph, b, oracle, results_equal)


MPD = 20037581.187 / 180.0


def stop_and_go(b, seed, stops_per_trace=3, max_stop=20, jitter_m=2.0):
    """Stops inserted into a batch: at a few points of each trace the vehicle
    stands for 2..max_stop one-second samples jittered by jitter_m (every
    later time shifted), so most of them fall within interpolation_distance
    of the stop's column."""
    rng = np.random.default_rng(seed)
    lat, lon, tm, acc, off = [], [], [], [], [0]
    for t in range(len(b["trace_off"]) - 1):
        a, e = int(b["trace_off"][t]), int(b["trace_off"][t + 1])
        stops = set(rng.choice(e - a, size=min(stops_per_trace, e - a), replace=False).tolist())
        shift = 0.0
        for i in range(a, e):
            lat.append(b["lat"][i])
            lon.append(b["lon"][i])
            tm.append(b["time"][i] + shift)
            acc.append(b["accuracy"][i])
            if i - a in stops:
                for _ in range(int(rng.integers(2, max_stop))):
                    shift += 1.0
                    dy, dx = rng.normal(0.0, jitter_m, 2)
                    la = float(b["lat"][i])
                    lat.append(la + dy / MPD)
                    lon.append(float(b["lon"][i]) + dx / (MPD * np.cos(np.radians(la))))
                    tm.append(b["time"][i] + shift)
                    acc.append(b["accuracy"][i])
        off.append(len(lat))
    return dict(trace_off=np.array(off, np.int64), lat=np.array(lat, np.float32), lon=np.array(lon, np.float32),
                time=np.array(tm, np.float64), accuracy=np.array(acc, np.float32))


@pytest.mark.parametrize("kind", ["dense", "stop_and_go", "long_stop_and_go"])
def test_interpolated_points(small_graph, oracle, results_equal, batch_path, kind):
    # SURVEY Appendix B / README.md:162-163: interpolated points are placed on
    # the matched route and the segment shape indices are the last point
    # before/at each boundary (DESIGN.md §3 rule 7) -- bit-identical to the
    # oracle, with the indices landing on interpolated points
    if kind == "dense":
        # one-second sampling: a local street's 8-11 m per step with 5 m noise
        b = synth.make_traces(small_graph, 150, 100, interval_s=1.0, noise_sigma_m=5.0, accuracy=10.0, seed=41)
    elif kind == "stop_and_go":
        b = stop_and_go(synth.make_traces(small_graph, 150, 60, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0,
                                          seed=43), seed=44)
    else:
        # traces beyond the segment kernel's LDS plans (the serial walk)
        b = stop_and_go(synth.make_traces(small_graph, 12, 240, interval_s=2.0, noise_sigma_m=5.0, accuracy=10.0,
                                          seed=45), seed=46, stops_per_trace=8)
        assert np.diff(b["trace_off"]).max() > 256
    res, orc = _run_both(small_graph, b, oracle, results_equal)
    ip = orc["ipos"]
    P = len(b["lat"])
    assert (ip >= 0).sum() > P // 50
    # shape indices are trace-relative: map them to batch points
    tr, segs = orc["traces"], orc["segments"]
    landed = 0
    for t in range(len(tr)):
        a, c = int(tr["seg_off"][t]), int(tr["seg_cnt"][t])
        base = int(b["trace_off"][t])
        for f in ("begin_shape_index", "end_shape_index"):
            landed += int((ip[base + segs[f][a:a + c]] >= 0).sum())
    assert landed > 20


def test_interpolated_points_hand_road(tmp_path, oracle, results_equal):
    # the hand-built road of tests/test_interp.py, on the GPU
    import handgraph
    path, _ = handgraph.straight_road(str(tmp_path / "road.otmg"), lat=40.0, n_nodes=5)
    traces = [[(0.0002, 0.0), (0.00025, 1.0), (0.00022, 2.0), (0.0003, 3.0), (0.0011, 10.0), (0.0021, 20.0)],
              [(0.0005, 0.0), (0.0005, 5.0), (0.0005, 10.0), (0.0005, 15.0), (0.0015, 25.0)],
              [(0.0002, 0.0), (0.00028, 1.0), (0.0012, 30.0), (0.0022, 40.0), (0.0032, 50.0)],
              # rule 4's stay: a probe behind the previous column on the same edge (test_interp.py)
              [(0.0002, 0.0), (0.0006, 5.0), (0.00045, 10.0), (0.0009, 15.0), (0.0014, 20.0)],
              [(0.0002, 0.0), (0.0006, 5.0), (0.00045, 10.0)]]
    lon = np.concatenate([np.array([p[0] for p in t], np.float32) for t in traces])
    tm = np.concatenate([np.array([p[1] for p in t], np.float64) for t in traces])
    off = np.concatenate([[0], np.cumsum([len(t) for t in traces])]).astype(np.int64)
    b = dict(trace_off=off, lat=np.full(len(lon), 40.0, np.float32), lon=lon, time=tm,
             accuracy=np.full(len(lon), 5.0, np.float32))
    res, orc = _run_both(path, b, oracle, results_equal)
    s = res.segments
    assert list(s["begin_shape_index"][:3]) == [0, 3, 4]
    assert list(s["end_shape_index"][:3]) == [3, 4, 5]
    assert res.traces["shape_used"][2] == 1
    assert res.traces["seg_cnt"][3] == 2 and res.traces["seg_cnt"][4] == 1


def test_empty_batch(small_graph):
    with Engine(graph_path=small_graph) as eng:
        r = eng.match(dict(trace_off=np.zeros(1, np.int64), lat=np.zeros(0, np.float32),
                           lon=np.zeros(0, np.float32), time=np.zeros(0), accuracy=np.zeros(0, np.float32)))
        assert len(r.traces) == 0 and len(r.segments) == 0


def test_deterministic_repeat(small_graph):
    b = synth.make_traces(small_graph, 100, 100, seed=13)
    with Engine(graph_path=small_graph) as eng:
        r1 = eng.match(b)
        r2 = eng.match(b)
    for a, c in ((r1.traces, r2.traces), (r1.segments, r2.segments), (r1.reports, r2.reports)):
        assert a.tobytes() == c.tobytes()


def test_json_report_path_byte_equal(small_graph, oracle):
    b = synth.make_traces(small_graph, 40, 60, seed=17)
    bodies = []
    for t in range(40):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        bodies.append(encode_request("veh%d" % t, b["lat"][a:e], b["lon"][a:e], b["time"][a:e].astype(np.int64),
                                     b["accuracy"][a:e].astype(np.int32)))
    bodies += [b"", b"[]", b'{"uuid":"x","trace":[]}', b'{"uuid":"x","trace":[{"lat":1}]}',
               b'{"uuid":"x","trace":[{"lat":1},{"lon":2}]}']
    g = oracle.Graph(small_graph)
    with Engine(graph_path=small_graph) as eng:
        got = eng.report_batch(bodies)
        single = eng.report(bodies[0])
        for body, (code, resp) in zip(bodies, got):
            ecode, eresp = oracle.handle_request(g, body)
            assert (code, resp) == (ecode, eresp), body[:80]
        assert single == got[0]
        # Match JSON (valhalla.SegmentMatcher().Match equivalent)
        for body in bodies[:5]:
            assert eng.match_json(body) == oracle.match_json(g, body)
        # async submit/poll returns the same bodies
        for k, body in enumerate(bodies[:10]):
            eng.submit(body, k)
        seen = {}
        while len(seen) < 10:
            for tag, code, resp in eng.poll(64, 2000000):
                seen[tag] = (code, resp)
        for k in range(10):
            assert seen[k] == got[k]


@pytest.mark.parametrize("form", ["8", "16", "64"])
def test_viterbi_forms(small_graph, rural_graph, oracle, results_equal, monkeypatch, form):
    """K5's three forms (kernels.hip launch_viterbi: 8 or 16 lanes per trace,
    each handing what it cannot take to the next, and the wave form) on the
    same batches, every stage bit-identical to the oracle: long traces past
    the grouped forms' 128 points, columns wider than 8 and 16 candidates
    (a 120 m radius in the city), chain breaks (gaps past the breakage
    distance) and a sparse rural graph."""
    monkeypatch.setenv("OTM_VIT_FORM", form)
    b = synth.make_traces(small_graph, 300, 60, seed=29)
    _run_both(small_graph, b, oracle, results_equal, counters=False)
    wide = synth.make_traces(small_graph, 120, 50, interval_s=5.0, noise_sigma_m=25.0, accuracy=25.0, seed=31)
    _run_both(small_graph, wide, oracle, results_equal, meili=dict(search_radius=120.0, max_search_radius=120.0),
              counters=False)
    long_ = synth.make_traces(small_graph, 20, 300, interval_s=5.0, seed=37)
    _run_both(small_graph, long_, oracle, results_equal, counters=False)
    gaps = synth.make_traces(small_graph, 100, 40, interval_s=240.0, noise_sigma_m=15.0, accuracy=15.0, seed=41)
    _run_both(small_graph, gaps, oracle, results_equal, meili=dict(breakage_distance=800.0), counters=False)
    rural = synth.make_traces(rural_graph, 200, 60, interval_s=30.0, noise_sigma_m=50.0, accuracy=50.0, seed=43)
    _run_both(rural_graph, rural, oracle, results_equal, counters=False)


def test_histogram_matches_reports(small_graph):
    import torch
    b = synth.make_traces(small_graph, 300, 100, seed=23)
    with Engine(graph_path=small_graph) as eng:
        nseg = eng.graph_info()["segments"]
        h = torch.zeros(nseg * 16, dtype=torch.int32, device="cuda:0")
        eng.hist_bind(h, 16, 10.0)
        r = eng.match(b)
        eng.hist_bind(None, 0, 1.0)
        torch.cuda.synchronize()
        ok = (r.reports["flags"] & 1) == 0
        speed = r.reports["length"] / (r.reports["t1"] - r.reports["t0"]) * 3.6
        ok &= speed >= 0
        assert int(h.sum().item()) == int(ok.sum())


def test_clone_concurrent_batches_identical(small_graph):
    """otm_engine_clone: batches on a parent and its clone, issued from two
    host threads at once, give the same bytes as the parent alone."""
    import threading
    a = synth.make_traces(small_graph, 300, 60, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=51)
    b = synth.make_traces(small_graph, 250, 80, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=52)
    with Engine(graph_path=small_graph) as eng:
        ra = eng.match(a)
        want_a = [getattr(ra, k).tobytes() for k in ("traces", "segments", "reports", "way_ids")]
        rb = eng.match(b)
        want_b = [getattr(rb, k).tobytes() for k in ("traces", "segments", "reports", "way_ids")]
        cl = eng.clone()
        try:
            got = {}

            def run(e, batch, key):
                for _ in range(3):
                    r = e.match(batch)
                got[key] = [getattr(r, k).tobytes() for k in ("traces", "segments", "reports", "way_ids")]
            th = [threading.Thread(target=run, args=(eng, a, "a")), threading.Thread(target=run, args=(cl, b, "b"))]
            for t in th:
                t.start()
            for t in th:
                t.join()
            assert got["a"] == want_a and got["b"] == want_b
        finally:
            cl.close()


def test_fetch_is_idempotent(small_graph):
    """otm_fetch_results may be called again for the same batch (a host that
    re-reads, the bench's checks after its timed legs): same arrays."""
    b = synth.make_traces(small_graph, 120, 60, seed=57)
    with Engine(graph_path=small_graph) as eng:
        r1 = eng.match(b)
        r2 = eng.fetch()
        r3 = eng.fetch()
    for k in ("traces", "segments", "reports", "way_ids"):
        assert getattr(r1, k).tobytes() == getattr(r2, k).tobytes() == getattr(r3, k).tobytes(), k


@pytest.mark.parametrize("fast", ["1", "0"], ids=["dom_free_reader", "dom"])
def test_json_report_path_host_threads(small_graph, oracle, monkeypatch, fast):
    """otm_report_batch's parse / point extraction / response writing split over
    host threads (forced here with tiny chunks), with the Java bodies read by
    the DOM-free reader or by the DOM path (OTM_FAST_JSON=0): byte-equal to the
    oracle, in request order, malformed bodies included."""
    monkeypatch.setenv("OTM_FAST_JSON", fast)
    b = synth.make_traces(small_graph, 120, 40, seed=19)
    bodies = []
    for t in range(120):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        bodies.append(encode_request("car%d" % t, b["lat"][a:e], b["lon"][a:e], b["time"][a:e].astype(np.int64),
                                     b["accuracy"][a:e].astype(np.int32)))
        if t % 17 == 3:
            bodies.append(b'{"uuid":"x","trace":[{"lat":1}]}')
        if t % 23 == 5:
            bodies.append(b"[]")
    g = oracle.Graph(small_graph)
    monkeypatch.setenv("OTM_HOST_THREADS", "7")
    monkeypatch.setenv("OTM_HOST_CHUNK", "5")
    with Engine(graph_path=small_graph) as eng:
        got = eng.report_batch(bodies)
        for body, (code, resp) in zip(bodies, got):
            assert (code, resp) == oracle.handle_request(g, body), body[:80]
        monkeypatch.setenv("OTM_HOST_THREADS", "1")
        assert eng.report_batch(bodies) == got


def test_pinned_host_batch_copy_path(small_graph):
    """otm_match_soa from pinned host buffers (otm_host_alloc): the same
    results as from pageable numpy arrays."""
    import ctypes as C
    from reporter_amd import _lib
    L = _lib.lib()
    from reporter_amd.engine import Results
    b = synth.make_traces(small_graph, 5000, 60, seed=29)  # 300k points (> 2^18): the large-batch copy path
    with Engine(graph_path=small_graph) as eng:
        want = eng.match(b)
        want = [getattr(want, k).tobytes() for k in ("traces", "segments", "reports", "way_ids")]
        ptrs, keep = {}, []
        for k in ("trace_off", "lat", "lon", "time", "accuracy"):
            a = np.ascontiguousarray(b[k])
            p = L.otm_host_alloc(a.nbytes)
            assert p
            C.memmove(p, a.ctypes.data, a.nbytes)
            ptrs[k] = p
            keep.append(p)
        try:
            hb = _lib.Batch(len(b["trace_off"]) - 1, int(b["trace_off"][-1]), ptrs["trace_off"], ptrs["lat"],
                            ptrs["lon"], ptrs["time"], ptrs["accuracy"])
            r = _lib.Results()
            assert L.otm_match_soa(eng.h, C.byref(hb), C.byref(r)) == 0
            got = Results(r)
            assert [getattr(got, k).tobytes() for k in ("traces", "segments", "reports", "way_ids")] == want
        finally:
            for p in keep:
                L.otm_host_free(p)


@pytest.mark.parametrize("size", ["small", "large"])
def test_compact_host_batch(small_graph, oracle, results_equal, size):
    """otm_match_compact (int32 time deltas, int16 accuracies, widened on the
    device by k_expand_compact): the same results as otm_match_soa on the
    widened batch, for the one-DMA small path and the large copy path (> 2^18
    points), with empty and one-point traces and zero / negative / large
    accuracies; and through a multi-device engine (widened on the host)."""
    from reporter_amd.engine import compact_batch
    n = 5000 if size == "large" else 300
    b = synth.make_traces(small_graph, n, 60, seed=41)
    lat, lon, tm, acc = (list(b[k]) for k in ("lat", "lon", "time", "accuracy"))
    off = list(b["trace_off"])
    for la, lo, t, a in [([], [], [], []), ([lat[0]], [lon[0]], [tm[0] + 7], [0.0]),
                         ([lat[5], lat[6], lat[7]], [lon[5], lon[6], lon[7]], [tm[5], tm[5] + 4, tm[5] + 9],
                          [-1.0, 500.0, 32767.0])]:
        lat += la
        lon += lo
        tm += t
        acc += a
        off.append(off[-1] + len(la))
    b = dict(trace_off=np.array(off, np.int64), lat=np.array(lat, np.float32), lon=np.array(lon, np.float32),
             time=np.array(tm, np.float64), accuracy=np.array(acc, np.float32))
    cb = compact_batch(b)
    assert cb["time_delta"].dtype == np.int32 and cb["accuracy"].dtype == np.int16
    keys = ("traces", "segments", "reports", "way_ids")
    with Engine(graph_path=small_graph) as eng:
        want = eng.match(b)
        got = eng.match_compact(b)
        assert [getattr(got, k).tobytes() for k in keys] == [getattr(want, k).tobytes() for k in keys]
        npt.assert_array_equal(eng.debug("in_time")[:len(lat)], b["time"])
        npt.assert_array_equal(eng.debug("in_acc")[:len(lat)], b["accuracy"])
    if size == "small":
        orc = oracle.match_batch(oracle.Graph(small_graph), b, nthreads=4)
        results_equal(orc, want, "compact")
        with Engine(graph_path=small_graph, devices=[0, 0]) as grp:
            g = grp.match_compact(b)
            assert [getattr(g, k).tobytes() for k in keys] == [getattr(want, k).tobytes() for k in keys]
