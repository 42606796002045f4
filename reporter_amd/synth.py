"""Synthetic inputs -- harness tooling over libotmatch.

No Valhalla tiles or real probe data exist here, so every workload is a
seeded synthetic road network plus seeded probe traces:

  config 1  small extract (5 x 5 km), synthesize_gps-style traces (one point
            per edge end, stddev 0: py/generate_test_trace.py:31-73)
  config 2  city 20 x 20 km, 10k vehicles x 100 points, 5 s, sigma 15 m
  config 3  metro 100 x 100 km, 1M vehicles x 100 points (uuid-sharded)
  config 4  state 500 x 500 km highway-heavy, 30 s, sigma 50 m, radius 100 m
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
            meili=dict(search_radius=100.0, max_search_radius=100.0)),
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


def _dedup(seq):
    out = []
    for x in seq:
        if not out or out[-1] != x:
            out.append(x)
    return out


def _lcs(a, b):
    if not a or not b:
        return 0
    prev = [0] * (len(b) + 1)
    for x in a:
        cur = [0]
        for j, y in enumerate(b):
            cur.append(prev[j] + 1 if x == y else max(prev[j + 1], cur[j]))
        prev = cur
    return prev[-1]


def segment_agreement(graph_path, path_off, path_edges, results):
    """Implementation-independent accuracy of a matched batch against the
    generator's ground truth: per trace the OSMLR segment-id sequence the
    vehicle drove (segments of its true edges, consecutive repeats merged)
    against the matched one (segments with an id, in order).  Returns
    {"segment_id_agreement": sum LCS / sum max(len), "sequences_exact":
    fraction of traces whose sequences are equal, "traces": n}."""
    ids = segment_ids(graph_path)
    eseg = edge_segments(graph_path)
    tr = results.traces if hasattr(results, "traces") else results["traces"]
    segs = results.segments if hasattr(results, "segments") else results["segments"]
    lcs = den = exact = 0
    for t in range(len(tr)):
        e = path_edges[path_off[t]:path_off[t + 1]]
        sg = eseg[e]
        truth = _dedup(ids[sg[sg >= 0]].tolist())
        a, n = int(tr["seg_off"][t]), int(tr["seg_cnt"][t])
        m = segs["segment_id"][a:a + n]
        got = _dedup(m[m >= 0].astype(np.uint64).tolist())
        lcs += _lcs(truth, got)
        den += max(len(truth), len(got))
        exact += truth == got
    return {"segment_id_agreement": lcs / float(max(den, 1)), "sequences_exact": exact / float(max(len(tr), 1)),
            "traces": len(tr)}


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
