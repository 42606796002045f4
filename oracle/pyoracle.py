"""ctypes binding of the CPU oracle (oracle/build/libotm_oracle.so).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product never imports this module.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# OTM_ORACLE_LIB: another build of the same oracle (the ASan/UBSan one, tests/test_sanitizers.py)
LIB_PATH = os.environ.get("OTM_ORACLE_LIB") or os.path.join(_HERE, "build", "libotm_oracle.so")
KMAX = 32

SEGMENT_DTYPE = np.dtype([("segment_id", "<i8"), ("start_time", "<f8"), ("end_time", "<f8"), ("length", "<i4"),
                          ("queue_length", "<i4"), ("begin_shape_index", "<i4"), ("end_shape_index", "<i4"),
                          ("way_off", "<i4"), ("way_cnt", "<i4"), ("flags", "<u4"), ("pad", "<u4")])
REPORT_DTYPE = np.dtype([("id", "<i8"), ("next_id", "<i8"), ("t0", "<f8"), ("t1", "<f8"), ("length", "<i4"),
                         ("queue_length", "<i4"), ("flags", "<u4"), ("pad", "<u4")])
TRACE_DTYPE = np.dtype([(n, "<i4") for n in (
    "code", "error_kind", "seg_off", "seg_cnt", "rep_off", "rep_cnt", "shape_used", "successful_count",
    "unreported_count", "discontinuities", "invalid_speeds", "unassociated", "successful_length",
    "unreported_length")])
COUNTER_NAMES = ("points", "columns", "cells_visited", "cell_entries_scanned", "candidates", "searches", "nodes_settled",
                 "edges_relaxed", "transitions", "route_searches", "route_nodes_settled", "route_edges_relaxed",
                 "route_edges", "segments_out", "reports_out", "edges_projected", "edge_shape_points")


class Params(C.Structure):
    _fields_ = [("sigma_z", C.c_float), ("beta", C.c_float), ("max_route_distance_factor", C.c_float),
                ("breakage_distance", C.c_float), ("interpolation_distance", C.c_float),
                ("search_radius", C.c_float), ("max_search_radius", C.c_float), ("gps_accuracy", C.c_float),
                ("max_candidates", C.c_int), ("turn_penalty_factor", C.c_float)]


class ReportCfg(C.Structure):
    _fields_ = [("n_report", C.c_int), ("n_transition", C.c_int), ("report_levels", C.c_int64 * 32),
                ("transition_levels", C.c_int64 * 32), ("threshold_sec", C.c_double)]


class Counters(C.Structure):
    _fields_ = [(n, C.c_int64) for n in COUNTER_NAMES]


class Results(C.Structure):
    _fields_ = [("n_traces", C.c_int32), ("n_segments", C.c_int32), ("n_reports", C.c_int32),
                ("n_way_ids", C.c_int32), ("traces", C.c_void_p), ("segments", C.c_void_p),
                ("reports", C.c_void_p), ("way_ids", C.c_void_p), ("n_points", C.c_int64),
                ("ncand", C.c_void_p), ("cand_edge", C.c_void_p), ("cand_off", C.c_void_p),
                ("cand_emis", C.c_void_p), ("trans_off", C.c_void_p), ("trans", C.c_void_p),
                ("state", C.c_void_p), ("col_prev", C.c_void_p), ("route_dist", C.c_void_p),
                ("gc", C.c_void_p), ("counters", Counters), ("ipos", C.c_void_p)]


# The CPU baseline's build of the same sources (oracle/Makefile `native`:
# -O3 -march=x86-64-v4, AVX-512, for the GPU box's EPYC host); bench.py times it
# and checks its output against the portable build's, byte for byte.
NATIVE_LIB_PATH = os.path.join(_HERE, "build", "native", "libotm_oracle.so")

_lib = None
_native = None


def host_has_avx512():
    try:
        with open("/proc/cpuinfo") as f:
            flags = f.read()
        return all(x in flags for x in ("avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl"))
    except OSError:
        return False


def native_lib():
    """The baseline build when it exists and this host can run it, else None."""
    global _native
    if _native is None and os.path.exists(NATIVE_LIB_PATH) and host_has_avx512():
        _native = _declare(C.CDLL(NATIVE_LIB_PATH))
    return _native


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: run `make -C oracle` (%s missing)" % LIB_PATH)
        _lib = _declare(C.CDLL(LIB_PATH))
    return _lib


def _declare(L):
    L.orc_graph_load.restype = C.c_void_p
    L.orc_graph_load.argtypes = [C.c_char_p]
    L.orc_graph_free.argtypes = [C.c_void_p]
    L.orc_graph_count.restype = C.c_int64
    L.orc_graph_count.argtypes = [C.c_void_p, C.c_int]
    L.orc_params_default.argtypes = [C.POINTER(Params)]
    L.orc_report_cfg_default.argtypes = [C.POINTER(ReportCfg)]
    L.orc_cos_deg.restype = C.c_float
    L.orc_cos_deg.argtypes = [C.c_float]
    L.orc_match_batch.argtypes = [C.c_void_p, C.POINTER(Params), C.POINTER(ReportCfg), C.c_int32,
                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                  C.c_int, C.POINTER(Results)]
    L.orc_results_free.argtypes = [C.POINTER(Results)]
    for fn in ("orc_handle_request",):
        getattr(L, fn).argtypes = [C.c_void_p, C.POINTER(Params), C.POINTER(ReportCfg), C.c_char_p,
                                   C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.orc_match_json.argtypes = [C.c_void_p, C.POINTER(Params), C.c_char_p, C.c_size_t,
                                 C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.orc_report_segments.argtypes = [C.POINTER(ReportCfg), C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
                                      C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_void_p)]
    L.orc_handle_batch.argtypes = [C.c_void_p, C.POINTER(Params), C.POINTER(ReportCfg), C.c_int,
                                   C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_int,
                                   C.POINTER(C.c_int), C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.orc_json_redump.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.orc_decode_polyline6.restype = C.c_int64
    L.orc_decode_polyline6.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_int64]
    L.orc_free.argtypes = [C.c_void_p]
    return L


def _take(ptr, n):
    s = C.string_at(ptr, n)
    lib().orc_free(ptr)
    return s


def params(**kw):
    p = Params()
    lib().orc_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def report_cfg(report_levels=(0, 1), transition_levels=(0, 1), threshold_sec=15.0):
    c = ReportCfg()
    c.n_report = len(report_levels)
    c.n_transition = len(transition_levels)
    for i, v in enumerate(report_levels):
        c.report_levels[i] = v
    for i, v in enumerate(transition_levels):
        c.transition_levels[i] = v
    c.threshold_sec = float(threshold_sec)
    return c


def report_cfg_from_env(env):
    """make_thread_locals (py/reporter_service.py:51-62) over an env dict."""
    rl = [int(i) for i in env.get("REPORT_LEVELS", "0,1").split(",")]
    tl = [int(i) for i in env.get("TRANSITION_LEVELS", "0,1").split(",")]
    thr = 15.0
    t = env.get("THRESHOLD_SEC")
    if t:
        low = t.lower()
        if low in ("y", "yes", "t", "true", "on", "1"):
            thr = 1.0
        elif low in ("n", "no", "f", "false", "off", "0"):
            thr = 0.0
        else:
            raise ValueError("invalid truth value %r" % (t,))
    return report_cfg(rl, tl, thr)


class Graph(object):
    def __init__(self, path, L=None):
        self.path = path
        self.L = L or lib()
        self.h = self.L.orc_graph_load(path.encode())
        if not self.h:
            raise RuntimeError("oracle cannot load graph %s" % path)

    def close(self):
        if self.h:
            self.L.orc_graph_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


def _arr(ptr, dtype, n):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    buf = (C.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=n).copy()


def match_batch(graph, batch, p=None, rc=None, nthreads=1, keep_stages=False, L=None):
    """batch: dict of numpy arrays trace_off(i64), lat(f32), lon(f32), time(f64), accuracy(f32).
    L: another build of the oracle (native_lib()) for the graph's handle."""
    L = L or graph.L
    p = p or params()
    rc = rc or report_cfg()
    off = np.ascontiguousarray(batch["trace_off"], dtype=np.int64)
    lat = np.ascontiguousarray(batch["lat"], dtype=np.float32)
    lon = np.ascontiguousarray(batch["lon"], dtype=np.float32)
    tm = np.ascontiguousarray(batch["time"], dtype=np.float64)
    acc = np.ascontiguousarray(batch["accuracy"], dtype=np.float32)
    r = Results()
    rcode = L.orc_match_batch(graph.h, C.byref(p), C.byref(rc), len(off) - 1, off.ctypes.data,
                                  lat.ctypes.data, lon.ctypes.data, tm.ctypes.data, acc.ctypes.data, nthreads,
                                  1 if keep_stages else 0, C.byref(r))
    if rcode != 0:
        raise RuntimeError("orc_match_batch failed")
    out = {
        "traces": _arr(r.traces, TRACE_DTYPE, r.n_traces),
        "segments": _arr(r.segments, SEGMENT_DTYPE, r.n_segments),
        "reports": _arr(r.reports, REPORT_DTYPE, r.n_reports),
        "way_ids": _arr(r.way_ids, np.int64, r.n_way_ids),
        "counters": {n: getattr(r.counters, n) for n in COUNTER_NAMES},
    }
    if keep_stages:
        P = r.n_points
        out["ncand"] = _arr(r.ncand, np.int32, P)
        out["cand_edge"] = _arr(r.cand_edge, np.int32, P * KMAX)
        out["cand_off"] = _arr(r.cand_off, np.float32, P * KMAX)
        out["cand_emis"] = _arr(r.cand_emis, np.float32, P * KMAX)
        out["trans_off"] = _arr(r.trans_off, np.int64, P + 1)
        out["trans"] = _arr(r.trans, np.float32, int(out["trans_off"][-1]) if P else 0)
        out["state"] = _arr(r.state, np.int32, P)
        out["col_prev"] = _arr(r.col_prev, np.int32, P)
        out["route_dist"] = _arr(r.route_dist, np.float32, P)
        out["gc"] = _arr(r.gc, np.float32, P)
        out["ipos"] = _arr(r.ipos, np.float32, P)
    L.orc_results_free(C.byref(r))
    return out


def handle_request(graph, body, p=None, rc=None, path="/report"):
    p = p or params()
    rc = rc or report_cfg()
    if isinstance(body, str):
        body = body.encode("utf-8")
    out = C.c_void_p()
    n = C.c_size_t()
    code = lib().orc_handle_request(graph.h if graph is not None else None, C.byref(p), C.byref(rc), path.encode(),
                                    body, len(body), C.byref(out), C.byref(n))
    return code, _take(out, n.value).decode("utf-8")


def match_json(graph, req, p=None):
    p = p or params()
    if isinstance(req, str):
        req = req.encode("utf-8")
    out = C.c_void_p()
    n = C.c_size_t()
    code = lib().orc_match_json(graph.h, C.byref(p), req, len(req), C.byref(out), C.byref(n))
    return code, _take(out, n.value).decode("utf-8")


def report_segments(req, match_output, rc=None):
    rc = rc or report_cfg()
    if isinstance(req, str):
        req = req.encode("utf-8")
    if isinstance(match_output, str):
        match_output = match_output.encode("utf-8")
    out = C.c_void_p()
    n = C.c_size_t()
    err = C.c_void_p()
    code = lib().orc_report_segments(C.byref(rc), req, len(req), match_output, len(match_output), C.byref(out),
                                     C.byref(n), C.byref(err))
    body = _take(out, n.value).decode("utf-8")
    e = C.string_at(err).decode("utf-8")
    lib().orc_free(err)
    return code, body, e


def handle_batch(graph, bodies, p=None, rc=None, nthreads=1, L=None):
    """orc_handle_batch: JSON request bodies -> [(code, body bytes)] (request
    parse, match, report(), response writing), nthreads host threads."""
    L = L or graph.L
    p = p or params()
    rc = rc or report_cfg()
    n = len(bodies)
    arr = (C.c_char_p * n)(*bodies)
    lens = (C.c_size_t * n)(*[len(b) for b in bodies])
    codes = (C.c_int * n)()
    outs = (C.c_void_p * n)()
    olens = (C.c_size_t * n)()
    L.orc_handle_batch(graph.h, C.byref(p), C.byref(rc), n, arr, lens, nthreads, codes, outs, olens)
    res = []
    for i in range(n):
        s = C.string_at(outs[i], olens[i])
        L.orc_free(outs[i])
        res.append((codes[i], s))
    return res


class HandlerCtx(C.Structure):
    _fields_ = [("g", C.c_void_p), ("p", C.c_void_p), ("rc", C.c_void_p), ("nthreads", C.c_int)]


class BatcherHandler(object):
    """orc_batcher_handler + its context: the C oracle's /report handler as
    the native batcher's matcher callback (no Python per call).  `fn` is the
    callback's address, `ctx` the context's; keep this object alive while the
    batcher runs."""

    def __init__(self, graph, p=None, rc=None, nthreads=1):
        L = graph.L
        self._keep = (graph, p or params(), rc or report_cfg())
        self.ctx = HandlerCtx(graph.h, C.addressof(self._keep[1]), C.addressof(self._keep[2]), nthreads)
        self.fn = C.cast(L.orc_batcher_handler, C.c_void_p).value
        self.ctx_ptr = C.addressof(self.ctx)


def json_redump(s):
    if isinstance(s, str):
        s = s.encode("utf-8")
    out = C.c_void_p()
    n = C.c_size_t()
    ok = lib().orc_json_redump(s, len(s), C.byref(out), C.byref(n))
    return ok, _take(out, n.value).decode("utf-8")


def decode_polyline6(enc):
    b = enc.encode("ascii")
    n = lib().orc_decode_polyline6(b, len(b), None, 0)
    if n < 0:
        raise ValueError("truncated polyline")
    out = np.zeros(2 * max(n, 1), dtype=np.float64)
    lib().orc_decode_polyline6(b, len(b), out.ctypes.data, n)
    return [[float(out[2 * i]), float(out[2 * i + 1])] for i in range(n)]


def cos_deg(x):
    return lib().orc_cos_deg(x)
