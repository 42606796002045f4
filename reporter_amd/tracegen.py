"""Config-1 trace generation: restatement of py/generate_test_trace.py.

The reference builds a test trace by routing A->B on a live Valhalla (/route),
walking the route's edges (/trace_attributes) and synthesizing one GPS point
per edge end (synthesize_gps, py/generate_test_trace.py:31-73).  No Valhalla
service exists here, so routes come from our synthetic graph and the edges
list is built from the graph; `decode` and `synthesize_gps` themselves are
restated faithfully (pinned by tests/golden/{decode,synth}_cases.json).

Not restated (documented reference bugs): for stddev > 0 the
reference references an unimported `np` (:53) and scales the latitude sigma by
cos(degrees) as if radians (:57).  Benchmark noise comes from
reporter_amd.synth instead.
"""
import json

import numpy as np


def decode(encoded):
    """Polyline6 -> [[lon, lat], ...] (py/generate_test_trace.py:9-29)."""
    inv = 1.0 / 1e6
    decoded = []
    previous = [0, 0]
    i = 0
    while i < len(encoded):
        ll = [0, 0]
        for j in (0, 1):
            shift = 0
            byte = 0x20
            while byte >= 0x20:
                byte = ord(encoded[i]) - 63
                i += 1
                ll[j] |= (byte & 0x1f) << shift
                shift += 5
            ll[j] = previous[j] + (~(ll[j] >> 1) if ll[j] & 1 else (ll[j] >> 1))
            previous[j] = ll[j]
        decoded.append([float("%.6f" % (ll[1] * inv)), float("%.6f" % (ll[0] * inv))])
    return decoded


def encode(coords_lonlat):
    """[[lon, lat], ...] -> polyline6 (the encoder Valhalla's /route uses)."""
    out = []
    prev = [0, 0]
    for lon, lat in coords_lonlat:
        for j, v in enumerate((int(round(lat * 1e6)), int(round(lon * 1e6)))):
            d = v - prev[j]
            prev[j] = v
            d = ~(d << 1) if d < 0 else (d << 1)
            while d >= 0x20:
                out.append(chr((0x20 | (d & 0x1f)) + 63))
                d >>= 5
            out.append(chr(d + 63))
    return "".join(out)


def synthesize_gps(edges, shape, distribution="normal", stddev=0, uuid="999999", now=None):
    """py/generate_test_trace.py:31-73 for stddev == 0.  `now` pins the wall
    clock the reference reads with time.time() (:39)."""
    if stddev != 0:
        raise NotImplementedError("the reference's stddev > 0 path is broken (see module doc)")
    import time as _t
    json_dict = {"uuid": uuid, "trace": []}
    coords = decode(shape)
    max_coord = max([edge["end_shape_index"] for edge in edges])
    if max_coord >= len(coords):
        return None, None
    sttm = (now if now is not None else _t.time()) - 86400
    for i, edge in enumerate(edges):
        dist = edge["length"]
        speed = edge["speed"]
        begin = edge["begin_shape_index"]
        end = edge["end_shape_index"]
        lon, lat = coords[end]
        dur = dist / speed * 3600.0
        time = int(round(sttm + dur))
        if i == 0:
            st_lon, st_lat = coords[begin]
            json_dict["trace"].append({"lat": st_lat, "lon": st_lon, "time": sttm, "accuracy": min(5, stddev * 1e3)})
        json_dict["trace"].append({"lat": lat, "lon": lon, "time": time, "accuracy": min(5, stddev * 1e3)})
        sttm = time
    return json_dict


def _graph_arrays(graph_path):
    """Minimal .otmg reader for route building (harness only)."""
    import struct
    raw = np.fromfile(graph_path, dtype=np.uint8)
    fmt = "<8sII4i2iq3d4dQ"
    hsize = struct.calcsize(fmt)
    h = struct.unpack_from(fmt, raw, 0)
    secs = [struct.unpack_from("<QQ", raw, hsize + 16 * i) for i in range(23)]

    def sec(i, dt):
        o, n = secs[i]
        return np.frombuffer(raw, dtype=dt, count=n // np.dtype(dt).itemsize, offset=o)
    return dict(out_off=sec(2, np.int32), e_to=sec(4, np.int32), e_len=sec(5, np.float32),
                e_shape=sec(6, np.int32), e_flags=sec(10, np.uint8), e_speed=sec(12, np.float32),
                e_opp=sec(13, np.int32), s_lat=sec(14, np.float32), s_lon=sec(15, np.float32), n_edges=h[4])


def config1_requests(graph_path, n_traces=100, edges_per_trace=40, seed=1, now=1507000000.0):
    """Config 1: routes on the synthetic extract -> edges (as /trace_attributes
    would list them: length km, speed km/h, shape indices) -> synthesize_gps ->
    /report request bodies (json.dumps compact, as main() sends, :116)."""
    G = _graph_arrays(graph_path)
    rng = np.random.default_rng(seed)
    bodies = []
    ext = np.nonzero((G["e_flags"] & 1) == 0)[0]
    for t in range(n_traces):
        e = int(ext[rng.integers(len(ext))])
        coords = []
        edges = []
        for k in range(edges_per_trace):
            a, b = G["e_shape"][e], G["e_shape"][e + 1]
            pts = [[float(G["s_lon"][s]), float(G["s_lat"][s])] for s in range(a, b)]
            begin = max(len(coords) - 1, 0)
            coords.extend(pts if not coords else pts[1:])
            edges.append({"length": float(G["e_len"][e]) / 1000.0, "speed": float(G["e_speed"][e]),
                          "begin_shape_index": begin, "end_shape_index": len(coords) - 1})
            node = G["e_to"][e]
            outs = [o for o in range(G["out_off"][node], G["out_off"][node + 1]) if o != G["e_opp"][e]]
            e = int(outs[rng.integers(len(outs))]) if outs else int(G["e_opp"][e])
        shape = encode(coords)
        tr = synthesize_gps(edges, shape, uuid="cfg1_%d" % t, now=now)
        bodies.append(json.dumps(tr, separators=(",", ":")).encode())
    return bodies
