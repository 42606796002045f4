"""Synthetic inputs -- harness tooling over libotmatch.

No Valhalla tiles or real probe data exist here, so every workload is a
seeded synthetic road network plus seeded probe traces:

  config 1  small extract (5 x 5 km), synthesize_gps-style traces (one point
            per edge end, stddev 0: py/generate_test_trace.py:31-73)
  config 2  city 20 x 20 km, 10k vehicles x 100 points, 5 s, sigma 15 m
  config 3  metro 100 x 100 km, 1M vehicles x 100 points (uuid-sharded)
  config 4  state 500 x 500 km highway-heavy, 30 s, sigma 50 m, radius 200 m
"""
import ctypes as C
import os

import numpy as np

from . import _lib
from ._lib import lib

GRAPH_VERSION = 2  # OTMG_VERSION (include/otm_graph_format.h): cached graphs of another format are rebuilt

CONFIGS = {
    1: dict(graph=dict(width_m=5000, height_m=5000), traces=dict(n_vehicles=100, points_per_vehicle=60,
                                                                 interval_s=5.0, noise_sigma_m=0.0, accuracy=0.0)),
    2: dict(graph=dict(width_m=20000, height_m=20000), traces=dict(n_vehicles=10000, points_per_vehicle=100,
                                                                   interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0)),
    3: dict(graph=dict(width_m=100000, height_m=100000), traces=dict(n_vehicles=1000000, points_per_vehicle=100,
                                                                     interval_s=5.0, noise_sigma_m=15.0,
                                                                     accuracy=15.0)),
    4: dict(graph=dict(width_m=500000, height_m=500000, block_m=1200, jitter_m=150, arterial_every=4,
                       highway_every=8, complex_every=0, seg_max_m=5000),
            traces=dict(n_vehicles=100000, points_per_vehicle=100, interval_s=30.0, noise_sigma_m=50.0,
                        accuracy=50.0),
            # "wide search_radius" (BASELINE config 4): 4 sigma of the 50 m noise.  At 100 m, 4.7 % of
            # the columns had no candidate on their road and 12 % of the driven segments came out wrong
            # around them; at 200 m 0.008 % and 0.05 % (profiles/r04_accuracy/)
            meili=dict(search_radius=200.0, max_search_radius=200.0)),
}


def graph_params(**kw):
    p = _lib.SynthGraphParams()
    lib().otm_synth_graph_defaults(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def make_graph(path, **kw):
    p = graph_params(**kw)
    rc = lib().otm_synth_graph(C.byref(p), path.encode())
    if rc != 0:
        raise RuntimeError("otm_synth_graph failed: %s" % _lib.last_error())
    return path


def make_traces(graph_path, n_vehicles, points_per_vehicle, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0,
                t0=1500000000.0, seed=7, vehicle_offset=0, vehicle_ids=None):
    """-> dict of numpy arrays: trace_off, lat, lon, time, accuracy, true_edge, true_off.

    Vehicle v's stream depends only on (seed, global id), the global id being
    vehicle_offset + v or vehicle_ids[v]: uuid shards regenerate identically."""
    ids = None
    if vehicle_ids is not None:
        ids = np.ascontiguousarray(vehicle_ids, dtype=np.int32)
        n_vehicles = len(ids)
    tp = _lib.SynthTraceParams(n_vehicles, points_per_vehicle, interval_s, noise_sigma_m, accuracy, t0, seed,
                               vehicle_offset, ids.ctypes.data if ids is not None else None)
    P = n_vehicles * points_per_vehicle
    out = dict(trace_off=np.zeros(n_vehicles + 1, np.int64), lat=np.zeros(P, np.float32),
               lon=np.zeros(P, np.float32), time=np.zeros(P, np.float64), accuracy=np.zeros(P, np.float32),
               true_edge=np.zeros(P, np.int32), true_off=np.zeros(P, np.float32))
    rc = lib().otm_synth_traces(graph_path.encode(), C.byref(tp), out["trace_off"].ctypes.data,
                                out["lat"].ctypes.data, out["lon"].ctypes.data, out["time"].ctypes.data,
                                out["accuracy"].ctypes.data, out["true_edge"].ctypes.data,
                                out["true_off"].ctypes.data)
    if rc != 0:
        raise RuntimeError("otm_synth_traces failed: %s" % _lib.last_error())
    return out


def cached_graph(config, cache_dir=None):
    """Generate (once) the graph of a config under cache_dir; returns its path."""
    cache_dir = cache_dir or os.environ.get("OTM_CACHE", "/tmp/otm_cache")
    os.makedirs(cache_dir, exist_ok=True)
    g = CONFIGS[config]["graph"]
    tag = "_".join("%s%s" % (k, v) for k, v in sorted(g.items()))
    path = os.path.join(cache_dir, "cfg%d_v%d_%s.otmg" % (config, GRAPH_VERSION, tag))
    if not os.path.exists(path):
        tmp = path + ".%d.tmp" % os.getpid()
        make_graph(tmp, **g)
        os.replace(tmp, path)
    return path


def segment_ids(graph_path):
    """The graph's OSMLR segment ids (u64[n_segments], section OTMG_SEG_ID of
    include/otm_graph_format.h), in segment-index order: row i of a
    histogram is segment_ids(...)[i]."""
    import struct
    raw = np.fromfile(graph_path, dtype=np.uint8)
    hs = struct.calcsize("<8sII4i2iq3d4dQ")
    o, n = struct.unpack_from("<QQ", raw, hs + 16 * 17)  # OTMG_SEG_ID
    return np.frombuffer(raw, dtype=np.uint64, count=n // 8, offset=o).copy()


def edge_segments(graph_path):
    """Per edge: its OSMLR segment index (-1 none), section OTMG_EDGE_SEG."""
    import struct
    raw = np.fromfile(graph_path, dtype=np.uint8)
    hs = struct.calcsize("<8sII4i2iq3d4dQ")
    o, n = struct.unpack_from("<QQ", raw, hs + 16 * 8)  # OTMG_EDGE_SEG
    return np.frombuffer(raw, dtype=np.int32, count=n // 4, offset=o).copy()


def true_paths(graph_path, n_vehicles, points_per_vehicle, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0,
               t0=1500000000.0, seed=7, vehicle_offset=0, vehicle_ids=None):
    """Ground truth of make_traces (same arguments): (path_off [V+1], edges) --
    the edges each vehicle drove from its first probe to its last."""
    ids = None
    if vehicle_ids is not None:
        ids = np.ascontiguousarray(vehicle_ids, dtype=np.int32)
        n_vehicles = len(ids)
    tp = _lib.SynthTraceParams(n_vehicles, points_per_vehicle, interval_s, noise_sigma_m, accuracy, t0, seed,
                               vehicle_offset, ids.ctypes.data if ids is not None else None)
    off = np.zeros(n_vehicles + 1, np.int64)
    n = lib().otm_synth_true_paths(graph_path.encode(), C.byref(tp), off.ctypes.data, None, 0)
    if n < 0:
        raise RuntimeError("otm_synth_true_paths failed: %s" % _lib.last_error())
    edges = np.zeros(max(n, 1), np.int32)
    lib().otm_synth_true_paths(graph_path.encode(), C.byref(tp), off.ctypes.data, edges.ctypes.data, n)
    return off, edges[:n]


def true_paths_timed(graph_path, n_vehicles, points_per_vehicle, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0,
                     t0=1500000000.0, seed=7, vehicle_offset=0, vehicle_ids=None):
    """true_paths with the time each vehicle entered each path edge:
    (path_off, edges, enter_time)."""
    ids = None
    if vehicle_ids is not None:
        ids = np.ascontiguousarray(vehicle_ids, dtype=np.int32)
        n_vehicles = len(ids)
    tp = _lib.SynthTraceParams(n_vehicles, points_per_vehicle, interval_s, noise_sigma_m, accuracy, t0, seed,
                               vehicle_offset, ids.ctypes.data if ids is not None else None)
    off = np.zeros(n_vehicles + 1, np.int64)
    n = lib().otm_synth_true_paths_timed(graph_path.encode(), C.byref(tp), off.ctypes.data, None, None, 0)
    if n < 0:
        raise RuntimeError("otm_synth_true_paths_timed failed: %s" % _lib.last_error())
    edges = np.zeros(max(n, 1), np.int32)
    enter = np.zeros(max(n, 1), np.float64)
    lib().otm_synth_true_paths_timed(graph_path.encode(), C.byref(tp), off.ctypes.data, edges.ctypes.data,
                                     enter.ctypes.data, n)
    return off, edges[:n], enter[:n]


def _dedup(seq):
    out = []
    for x in seq:
        if not out or out[-1] != x:
            out.append(x)
    return out


def _lcs_pairs(a, b):
    """One LCS alignment of a and b as index pairs (i, j), increasing."""
    n, m = len(a), len(b)
    if n == 0 or m == 0:
        return []
    L = np.zeros((n + 1, m + 1), np.int32)
    for i in range(n - 1, -1, -1):
        for j in range(m - 1, -1, -1):
            L[i, j] = L[i + 1, j + 1] + 1 if a[i] == b[j] else max(L[i + 1, j], L[i, j + 1])
    out = []
    i = j = 0
    while i < n and j < m:
        if a[i] == b[j]:
            out.append((i, j))
            i += 1
            j += 1
        elif L[i + 1, j] >= L[i, j + 1]:
            i += 1
        else:
            j += 1
    return out


ERROR_CLASSES = ("start_missed", "start_extra", "end_missed", "end_extra", "dropped", "inserted_outlier",
                 "inserted_uturn", "inserted_other", "reverse", "swap")
INTERIOR_CLASSES = ("dropped", "inserted_outlier", "inserted_uturn", "inserted_other", "reverse", "swap")
END_CLASSES = ("start_missed", "start_extra", "end_missed", "end_extra")


def classify_sequences(T, G, twin, at_outlier=lambda k0, k1: False):
    """Where a matched segment sequence G departs from the driven one T.

    An LCS alignment pairs them; what it leaves unpaired is an error:
      start_* / end_*  before the first / after the last pair: the trace's
                       first / last partial segment, whose heading and extent
                       the trace does not observe past its end point;
      interior, between two pairs:
        dropped           driven segments with nothing matched in their place
        inserted_outlier  matched segments over points whose road had no
                          candidate within the search radius (at_outlier(k0,
                          k1): the points from G[k0]'s end to G[k1]'s start)
        inserted_uturn    onto the opposite direction of a neighbouring
                          segment and back (B, rev(B), B)
        inserted_other    any other matched segment nothing was driven for
        reverse           a matched segment the opposite of a driven one
        swap              otherwise (a parallel street, another route)
    twin: segment id -> ids of its opposite direction."""
    c = dict((k, 0) for k in ERROR_CLASSES)
    pairs = _lcs_pairs(T, G)
    c.update(truth=len(T), matched=len(G), no_overlap=0, paired=len(pairs))
    if not pairs:
        c["no_overlap"] = 1
        c["start_missed"] = len(T)
        c["start_extra"] = len(G)
        return c
    (i0, j0), (i1, j1) = pairs[0], pairs[-1]
    c["start_missed"], c["start_extra"] = i0, j0
    c["end_missed"], c["end_extra"] = len(T) - 1 - i1, len(G) - 1 - j1
    for (pa, pb), (qa, qb) in zip(pairs, pairs[1:]):
        miss = T[pa + 1:qa]
        extra = G[pb + 1:qb]
        if miss and extra:
            rev = sum(1 for x in extra if twin.get(x, set()) & set(miss))
            c["reverse"] += rev
            c["swap"] += max(len(miss), len(extra)) - rev
        elif miss:
            c["dropped"] += len(miss)
        elif extra:
            if at_outlier(pb, qb):
                c["inserted_outlier"] += len(extra)
            elif all(x in twin.get(G[pb], set()) | twin.get(G[qb], set()) | {G[pb], G[qb]} for x in extra):
                c["inserted_uturn"] += len(extra)
            else:
                c["inserted_other"] += len(extra)
    return c


def _graph_section(graph_path, k, dtype):
    import struct
    raw = np.fromfile(graph_path, dtype=np.uint8)
    hs = struct.calcsize("<8sII4i2iq3d4dQ")
    o, n = struct.unpack_from("<QQ", raw, hs + 16 * k)
    return np.frombuffer(raw, dtype=dtype, count=n // np.dtype(dtype).itemsize, offset=o).copy()


def outlier_points(graph_path, true_edge, ncand, cand_edge, cand_off, trace_off, gc, kmax=32):
    """Per point: True for an HMM column whose true edge had no candidate --
    neither an edge candidate on it nor a node candidate at one of its end
    nodes (the probe fell outside its road's search radius).  Candidates and
    gc from a matcher's stage outputs (the oracle's, keep_stages=True): a
    point is a column when it starts its trace or has gc > 0 (rule 1: an
    interpolated point has none, a column is >= interpolation_distance from
    the previous one)."""
    e_from = _graph_section(graph_path, 3, np.int32)  # OTMG_EDGE_FROM
    e_to = _graph_section(graph_path, 4, np.int32)    # OTMG_EDGE_TO
    P = len(true_edge)
    ce = np.asarray(cand_edge).reshape(P, kmax)
    co = np.asarray(cand_off).reshape(P, kmax)
    valid = np.arange(kmax)[None, :] < np.asarray(ncand)[:, None]
    te = np.asarray(true_edge)[:, None]
    on_edge = (ce == te) & (co > 0)
    cf = e_from[np.clip(ce, 0, len(e_from) - 1)]
    at_node = (co == 0) & ((cf == e_from[te]) | (cf == e_to[te]))
    col = np.asarray(gc) > 0
    col[np.asarray(trace_off)[:-1][np.diff(trace_off) > 0]] = True
    return col & ~np.any(valid & (on_edge | at_node), axis=1)


def segment_agreement(graph_path, path_off, path_edges, results, trace_off=None, outlier=None, per_trace=None):
    """Implementation-independent accuracy of a matched batch against the
    generator's ground truth: per trace the OSMLR segment-id sequence the
    vehicle drove (segments of its true edges, consecutive repeats merged)
    against the matched one (segments with an id, in order).  Returns
    {"segment_id_agreement": sum LCS / sum max(len), "sequences_exact":
    fraction of traces whose sequences are equal, "traces": n, "breakdown":
    the error classes of classify_sequences summed over traces, with
    "interior_agreement" = 1 - interior errors / driven segments and
    "end_share" = the start/end errors' share of all errors}.  outlier (per
    point, outlier_points) and trace_off attribute insertions to probes
    outside their road's radius; per_trace (a list) receives each trace's
    classes."""
    ids = segment_ids(graph_path)
    eseg = edge_segments(graph_path)
    eopp = _graph_section(graph_path, 13, np.int32)  # OTMG_EDGE_OPP
    twin = {}
    for e in np.nonzero((eseg >= 0) & (eopp >= 0))[0]:
        o = eopp[e]
        if eseg[o] >= 0:
            twin.setdefault(int(ids[eseg[e]]), set()).add(int(ids[eseg[o]]))
    tr = results.traces if hasattr(results, "traces") else results["traces"]
    segs = results.segments if hasattr(results, "segments") else results["segments"]
    lcs = den = exact = 0
    tot = dict((k, 0) for k in ERROR_CLASSES)
    tot.update(truth=0, matched=0, no_overlap=0, paired=0)
    for t in range(len(tr)):
        e = path_edges[path_off[t]:path_off[t + 1]]
        sg = eseg[e]
        truth = _dedup(ids[sg[sg >= 0]].tolist())
        a, n = int(tr["seg_off"][t]), int(tr["seg_cnt"][t])
        m = segs["segment_id"][a:a + n].astype(np.int64)
        bsi = segs["begin_shape_index"][a:a + n]
        esi = segs["end_shape_index"][a:a + n]
        got, rng = [], []
        for x, bi, ei in zip(m.tolist(), bsi.tolist(), esi.tolist()):
            if x < 0:
                continue
            if got and got[-1] == x:
                rng[-1][1] = ei
            else:
                got.append(x)
                rng.append([bi, ei])
        at = (lambda k0, k1: False)
        if outlier is not None and trace_off is not None:
            p0 = int(trace_off[t])
            at = (lambda k0, k1, p0=p0, rng=rng: bool(outlier[p0 + rng[k0][1]:p0 + rng[k1][0] + 1].any()))
        c = classify_sequences(truth, got, twin, at)
        if per_trace is not None:
            per_trace.append(c)
        for k, v in c.items():
            tot[k] += v
        lcs += c["paired"]
        den += max(len(truth), len(got))
        exact += truth == got
    interior = sum(tot[k] for k in INTERIOR_CLASSES)
    ends = sum(tot[k] for k in END_CLASSES)
    driven = max(tot["truth"], 1)
    bd = dict(tot)
    bd.update(driven_segments=tot["truth"], interior_errors=interior, end_errors=ends,
              interior_agreement=1.0 - interior / float(driven),
              interior_agreement_outside_outliers=1.0 - (interior - tot["inserted_outlier"]) / float(driven),
              end_share=ends / float(max(ends + interior, 1)))
    if outlier is not None:
        bd["outlier_points"] = int(np.asarray(outlier).sum())
    return {"segment_id_agreement": lcs / float(max(den, 1)), "sequences_exact": exact / float(max(len(tr), 1)),
            "traces": len(tr), "breakdown": bd}


def true_segments(graph_path, path_off, path_edges, enter, last_time):
    """Per trace, the segment list the vehicle drove as a Match output would
    give it (the grouping and validity rules of DESIGN.md §3 rule 7, on the
    true route with its true times): consecutive path edges of one OSMLR
    segment (increasing position) or one run of unassociated edges of one
    internal flag form a segment; its start time is valid when the vehicle
    entered the segment's first edge after the trace began (the first path
    edge was entered before the first probe), its end time when it left the
    segment's last edge before the trace ended (the last path edge is left
    after the last probe); length only when both are.  Returns a list of
    lists of dicts (the Match JSON's segment objects)."""
    eseg = _graph_section(graph_path, 8, np.int32)       # OTMG_EDGE_SEG
    epos = _graph_section(graph_path, 9, np.int32)       # OTMG_EDGE_SEG_POS
    eflg = _graph_section(graph_path, 10, np.uint8)      # OTMG_EDGE_FLAGS
    gid = _graph_section(graph_path, 17, np.uint64)      # OTMG_SEG_ID
    glen = _graph_section(graph_path, 18, np.float32)    # OTMG_SEG_LEN
    out = []
    for t in range(len(path_off) - 1):
        a, e = int(path_off[t]), int(path_off[t + 1])
        E = path_edges[a:e]
        T = enter[a:e]
        m = len(E)
        segs = []
        i = 0
        while i < m:
            j = i
            while j + 1 < m:
                x, y = int(E[j]), int(E[j + 1])
                if eseg[y] >= 0:
                    join = eseg[x] == eseg[y] and epos[y] == epos[x] + 1
                else:
                    join = eseg[x] < 0 and ((eflg[x] ^ eflg[y]) & 1) == 0
                if not join:
                    break
                j += 1
            f, l = int(E[i]), int(E[j])
            sv = i > 0
            ev = j < m - 1
            d = {}
            if eseg[f] >= 0:
                sv = sv and bool(eflg[f] & 2)
                ev = ev and bool(eflg[l] & 4)
                d["segment_id"] = int(gid[eseg[f]])
                d["length"] = int(np.floor(float(glen[eseg[f]]) + 0.5)) if (sv and ev) else -1
                d["internal"] = False
            else:
                d["length"] = -1
                d["internal"] = bool(eflg[f] & 1)
            d["start_time"] = float(T[i]) if sv else -1
            d["end_time"] = float(T[j + 1]) if ev else -1
            d.update(queue_length=0, begin_shape_index=0, end_shape_index=0, way_ids=[])
            segs.append(d)
            i = j + 1
        out.append(segs)
    return out


REPORT_ERROR_CLASSES = ("start_missed", "start_extra", "end_missed", "end_extra", "interior_missed",
                        "interior_extra")


def report_agreement(graph_path, path_off, path_edges, enter, trace_off, time, results):
    """What the datastore receives, against the ground truth: per trace, the
    reports report() (py/reporter_service.py:110-196, the product's host
    restatement pinned by the reference's recorded cases) emits for the driven
    route with its true times (true_segments), against the matched batch's
    reports.  Reports pair up by an LCS over (id, next_id); unpaired ones
    before the first or after the last pair are start / end errors, the rest
    interior.  For the pairs: |t0 - true t0|, |t1 - true t1| (s) and the
    relative error of the reported speed length / (t1 - t0)."""
    import json as _json

    from .engine import report_segments
    truth = true_segments(graph_path, path_off, path_edges, enter, None)
    tr = results.traces if hasattr(results, "traces") else results["traces"]
    reps = results.reports if hasattr(results, "reports") else results["reports"]
    c = dict((k, 0) for k in REPORT_ERROR_CLASSES)
    n_truth = n_match = paired = den = exact = 0
    dt0, dt1, dsp = [], [], []
    for t in range(len(tr)):
        p1 = int(trace_off[t + 1]) - 1
        tl = float(time[p1])
        ts = int(tl) if tl == int(tl) else repr(tl)
        body = '{"uuid":"x","trace":[{"lat":0,"lon":0,"time":%s,"accuracy":5},{"lat":0,"lon":0,"time":%s,' \
               '"accuracy":5}]}' % (ts, ts)
        code, resp = report_segments(body, _json.dumps({"segments": truth[t]}, separators=(",", ":")))
        want = _json.loads(resp).get("datastore", {}).get("reports", []) if code == 200 else []
        a, n = int(tr["rep_off"][t]), int(tr["rep_cnt"][t])
        got = reps[a:a + n]
        kw = [(int(r["id"]), int(r.get("next_id", -1))) for r in want]
        kg = [(int(x), int(y)) for x, y in zip(got["id"].tolist(), got["next_id"].tolist())]
        pairs = _lcs_pairs(kw, kg)
        n_truth += len(kw)
        n_match += len(kg)
        paired += len(pairs)
        den += max(len(kw), len(kg))
        exact += kw == kg
        if not pairs:
            c["start_missed"] += len(kw)
            c["start_extra"] += len(kg)
            continue
        (i0, j0), (i1, j1) = pairs[0], pairs[-1]
        c["start_missed"] += i0
        c["start_extra"] += j0
        c["end_missed"] += len(kw) - 1 - i1
        c["end_extra"] += len(kg) - 1 - j1
        for (pa, pb), (qa, qb) in zip(pairs, pairs[1:]):
            c["interior_missed"] += qa - pa - 1
            c["interior_extra"] += qb - pb - 1
        for i, j in pairs:
            w, g = want[i], got[j]
            dt0.append(abs(float(g["t0"]) - float(w["t0"])))
            dt1.append(abs(float(g["t1"]) - float(w["t1"])))
            vw = float(w["length"]) / max(float(w["t1"]) - float(w["t0"]), 1e-9)
            vg = float(g["length"]) / max(float(g["t1"]) - float(g["t0"]), 1e-9)
            dsp.append(abs(vg - vw) / max(vw, 1e-9))
    q = lambda xs, f: float(np.percentile(xs, f)) if xs else None  # noqa: E731
    interior = c["interior_missed"] + c["interior_extra"]
    return {"report_agreement": paired / float(max(den, 1)), "traces_exact": exact / float(max(len(tr), 1)),
            "truth_reports": n_truth, "matched_reports": n_match, "paired": paired,
            "interior_error_rate": interior / float(max(n_truth, 1)),
            "errors": c,
            "t0_abs_error_s": {"p50": q(dt0, 50), "p90": q(dt0, 90), "max": max(dt0) if dt0 else None},
            "t1_abs_error_s": {"p50": q(dt1, 50), "p90": q(dt1, 90), "max": max(dt1) if dt1 else None},
            "speed_rel_error": {"p50": q(dsp, 50), "p90": q(dsp, 90), "p99": q(dsp, 99),
                                "within_1e-3": float(np.mean([x <= 1e-3 for x in dsp])) if dsp else None,
                                "within_5pct": float(np.mean([x <= 0.05 for x in dsp])) if dsp else None}}


def slice_batch(b, t0, t1):
    """Traces [t0, t1) of a batch as a new batch (offsets rebased)."""
    a, e = int(b["trace_off"][t0]), int(b["trace_off"][t1])
    out = {k: b[k][a:e] for k in ("lat", "lon", "time", "accuracy", "true_edge", "true_off") if k in b}
    out["trace_off"] = b["trace_off"][t0:t1 + 1] - a
    return out


def shard_vehicle_ids(n_per_rank, rank, world, prefix="veh"):
    """Global vehicle ids whose uuid ("veh<id>") lands on `rank` under Kafka's
    murmur2 key partitioner -- the uuid sharding of SURVEY.md §8(e)."""
    from .engine import murmur2_partition
    out = []
    v = 0
    while len(out) < n_per_rank:
        if world == 1 or murmur2_partition("%s%d" % (prefix, v), world) == rank:
            out.append(v)
        v += 1
    return np.array(out, np.int32)
