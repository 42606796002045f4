"""Engine: one MI355X, its HBM-resident road graph, the /report hot path.

Python face of libotmatch.so's C ABI (include/otmatch.h).  Mirrors the
reference's matcher interface (py/reporter_service.py): Engine.report(body)
answers like SegmentMatcherHandler.handle_request (:218-240) and
Engine.match_json(body) like valhalla.SegmentMatcher().Match (:112); the
binary entry points (match, match_device) are the benchmark path.
"""
import ctypes as C
import json
import os
import tempfile

import numpy as np

from . import _lib
from ._lib import lib, take


class OtmError(RuntimeError):
    pass


def _check(rc):
    if rc != _lib.OTM_OK:
        raise OtmError("libotmatch error %d: %s" % (rc, _lib.last_error()))


def write_config(path, graph_path, index_radius_m=None, grid_mult=None, trans_lanes=None, index_near_m=None,
                 **meili):
    """Write an engine config: {"otm":{"graph":...,"index_radius_m":R},"meili":{"default":{...}}}.
    index_near_m: the near indexes' radii (a list; [] for none; default a
    fraction of the index radius, engine.cpp build_index)."""
    otm = {"graph": os.path.abspath(graph_path)}
    if index_radius_m is not None:
        otm["index_radius_m"] = index_radius_m
    if index_near_m is not None:
        otm["index_near_m"] = list(index_near_m)
    if grid_mult is not None:
        otm["grid_mult"] = grid_mult
    if trans_lanes is not None:
        otm["trans_lanes"] = trans_lanes
    cfg = {"otm": otm, "meili": {"default": meili}}
    with open(path, "w") as f:
        json.dump(cfg, f)
    return path


def compact_batch(batch):
    """A batch narrowed to otm_batch_compact (the Java host's Point types):
    int64 time base per trace (its first time), int32 time deltas, int16
    accuracies.  Raises ValueError when a time is not a whole number of
    seconds, a delta leaves int32 or an accuracy leaves int16 (such a batch
    goes through Engine.match)."""
    off = np.ascontiguousarray(batch["trace_off"], dtype=np.int64)
    tm = np.asarray(batch["time"], dtype=np.float64)
    acc = np.asarray(batch["accuracy"], dtype=np.float32)
    ti = tm.astype(np.int64)
    if not np.array_equal(ti.astype(np.float64), tm):
        raise ValueError("compact batches carry whole-second times")
    ia = acc.astype(np.int64)
    if not np.array_equal(ia.astype(np.float32), acc) or (len(ia) and (ia.min() < -32768 or ia.max() > 32767)):
        raise ValueError("compact batches carry int16 accuracies")
    nt = len(off) - 1
    lens = np.diff(off)
    base = np.zeros(nt, dtype=np.int64)
    nz = lens > 0
    base[nz] = ti[off[:-1][nz]]
    delta = ti - np.repeat(base, lens)
    if len(delta) and (delta.min() < -2**31 or delta.max() >= 2**31):
        raise ValueError("a trace's times span more than int32 seconds")
    return {"trace_off": off, "time_base": base,
            "lat": np.ascontiguousarray(batch["lat"], dtype=np.float32),
            "lon": np.ascontiguousarray(batch["lon"], dtype=np.float32),
            "time_delta": delta.astype(np.int32), "accuracy": ia.astype(np.int16)}


class RequestArena(object):
    """Request bodies written back to back into library-owned page-locked
    memory (otm_request_arena_alloc), as the Java host writes its
    body.getBytes(ISO_8859_1) into a MemorySegment over the arena; pass it to
    Engine.report_batch / submit_batch in place of the bodies."""

    def __init__(self, bodies):
        bs = [b.encode("utf-8") if isinstance(b, str) else b for b in bodies]
        self.n = len(bs)
        total = sum(len(b) for b in bs)
        self.base = lib().otm_request_arena_alloc(max(total, 1))
        if not self.base:
            raise OtmError("otm_request_arena_alloc: %s" % _lib.last_error())
        blob = b"".join(bs)
        C.memmove(self.base, blob, len(blob))
        offs = np.zeros(self.n + 1, dtype=np.int64)
        np.cumsum([len(b) for b in bs], out=offs[1:])
        self.ptrs = (C.c_void_p * self.n)(*[self.base + int(o) for o in offs[:-1]])
        self.ptrs = C.cast(self.ptrs, C.POINTER(C.c_char_p))
        self.lens = (C.c_size_t * self.n)(*[len(b) for b in bs])
        self.bytes = total

    def release(self):
        if self.base:
            _check(lib().otm_request_arena_release(self.base))
            self.base = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.release()


class Results(object):
    """Host copy of one batch's results (numpy structured arrays)."""

    def __init__(self, r):
        self.traces = _lib.as_array(r.traces, _lib.TRACE_DTYPE, r.n_traces)
        self.segments = _lib.as_array(r.segments, _lib.SEGMENT_DTYPE, r.n_segments)
        self.reports = _lib.as_array(r.reports, _lib.REPORT_DTYPE, r.n_reports)
        self.way_ids = _lib.as_array(r.way_ids, np.int64, r.n_way_ids)


class Engine(object):
    def __init__(self, config_path=None, graph_path=None, device=0, index_radius_m=None, grid_mult=None,
                 trans_lanes=None, devices=None, index_near_m=None, **meili):
        """Either a config file (valhalla.Configure-style) or a graph path.
        devices=[d0, d1, ...] makes a multi-device engine (otm_engine_create
        with ndev > 1): traces go to member murmur2(uuid) % ndev."""
        L = lib()
        self._tmp = None
        if config_path is None:
            if graph_path is None:
                raise ValueError("config_path or graph_path required")
            fd, self._tmp = tempfile.mkstemp(suffix=".json", prefix="otm_cfg_")
            os.close(fd)
            config_path = write_config(self._tmp, graph_path, index_radius_m=index_radius_m, grid_mult=grid_mult,
                                       trans_lanes=trans_lanes, index_near_m=index_near_m, **meili)
        h = C.c_void_p()
        devs = list(devices) if devices is not None else [device]
        dev = (C.c_int * len(devs))(*devs)
        rc = L.otm_engine_create(config_path.encode(), dev, len(devs), C.byref(h))
        if rc != _lib.OTM_OK:
            raise OtmError("otm_engine_create failed (%d): %s" % (rc, _lib.last_error()))
        self.h = h
        self.device = devs[0]
        self.devices = devs

    def members(self):
        """Member count: ndev of a multi-device engine, else 1."""
        return lib().otm_engine_members(self.h)

    def member(self, i):
        """Member i of a multi-device engine as an Engine view (owned by self:
        do not close it; it lives as long as self)."""
        h = lib().otm_engine_member(self.h, i)
        if not h:
            raise OtmError("no member %d" % i)
        e = Engine.__new__(Engine)
        e._tmp = None
        e.h = C.c_void_p(h)
        e.device = self.devices[i] if len(self.devices) > 1 else self.device
        e.parent = self
        e._view = True
        return e

    def clone(self):
        """A second batch context on this GPU sharing the graph and index
        (otm_engine_clone): its own stream and buffers, so batches on the two
        run concurrently from different host threads.  Close it before self."""
        h = C.c_void_p()
        rc = lib().otm_engine_clone(self.h, C.byref(h))
        if rc != _lib.OTM_OK:
            raise OtmError("otm_engine_clone failed (%d): %s" % (rc, _lib.last_error()))
        e = Engine.__new__(Engine)
        e._tmp = None
        e.h = h
        e.device = self.device
        e.parent = self
        return e

    def close(self):
        if getattr(self, "_view", False):
            self.h = None  # a member view: its group owns it
        if getattr(self, "h", None):
            lib().otm_engine_destroy(self.h)
            self.h = None
        if getattr(self, "_tmp", None):
            try:
                os.unlink(self._tmp)
            except OSError:
                pass
            self._tmp = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------ request level
    def report(self, body):
        """-> (http_code, body_str), exactly as reporter_service.py answers /report."""
        b = body.encode("utf-8") if isinstance(body, str) else body
        out = C.c_void_p()
        n = C.c_size_t()
        code = lib().otm_report(self.h, b, len(b), C.byref(out), C.byref(n))
        return code, take(out, n.value).decode("utf-8")

    def report_batch(self, bodies):
        """otm_report_batch over request bodies (bytes / str), or over a
        RequestArena's bodies (sent to HBM straight from the arena)."""
        if isinstance(bodies, RequestArena):
            n, arr, lens = bodies.n, bodies.ptrs, bodies.lens
        else:
            bs = [b.encode("utf-8") if isinstance(b, str) else b for b in bodies]
            n = len(bs)
            arr = (C.c_char_p * n)(*bs)
            lens = (C.c_size_t * n)(*[len(b) for b in bs])
        outs = (C.c_void_p * n)()
        olens = (C.c_size_t * n)()
        codes = (C.c_int * n)()
        _check(lib().otm_report_batch(self.h, n, arr, lens, outs, olens, codes))
        return [(codes[i], take(outs[i], olens[i]).decode("utf-8")) for i in range(n)]

    def match_json(self, body):
        b = body.encode("utf-8") if isinstance(body, str) else body
        out = C.c_void_p()
        n = C.c_size_t()
        code = lib().otm_match_json(self.h, b, len(b), C.byref(out), C.byref(n))
        return code, take(out, n.value).decode("utf-8")

    def report_segments(self, body, match_output):
        return report_segments(body, match_output, self)

    def report_segments_device(self, pairs):
        """report() on the GPU (k_report) over [(request body, Match output)]
        -> [(code, body)]; code 0 where a Match output does not fit the typed
        records (otm_report_segments_device)."""
        enc = lambda x: x.encode("utf-8") if isinstance(x, str) else x  # noqa: E731
        rq = [enc(a) for a, _ in pairs]
        mo = [enc(b) for _, b in pairs]
        n = len(pairs)
        outs = (C.c_void_p * n)()
        olens = (C.c_size_t * n)()
        codes = (C.c_int * n)()
        _check(lib().otm_report_segments_device(self.h, n, (C.c_char_p * n)(*rq), (C.c_size_t * n)(*map(len, rq)),
                                                (C.c_char_p * n)(*mo), (C.c_size_t * n)(*map(len, mo)), outs, olens,
                                                codes))
        return [(codes[i], take(outs[i], olens[i]).decode("utf-8")) for i in range(n)]

    def submit(self, body, tag):
        b = body.encode("utf-8") if isinstance(body, str) else body
        _check(lib().otm_submit(self.h, b, len(b), tag))

    def submit_batch(self, bodies, tags):
        """otm_submit_batch: many requests in one call (in order); a
        RequestArena's bodies are referenced, not copied."""
        if isinstance(bodies, RequestArena):
            n, arr, lens = bodies.n, bodies.ptrs, bodies.lens
        else:
            bs = [b.encode("utf-8") if isinstance(b, str) else b for b in bodies]
            n = len(bs)
            arr = (C.c_char_p * n)(*bs)
            lens = (C.c_size_t * n)(*[len(b) for b in bs])
        tg = (C.c_uint64 * n)(*tags)
        _check(lib().otm_submit_batch(self.h, n, arr, lens, tg))

    def poll(self, max_results=1024, timeout_us=0):
        res = (_lib.Result * max_results)()
        n = lib().otm_poll(self.h, res, max_results, timeout_us)
        if n < 0:
            _check(n)
        return [(res[i].tag, res[i].code, take(res[i].body, res[i].body_len).decode("utf-8")) for i in range(n)]

    # ------------------------------------------------------------ binary level
    def match(self, batch):
        """Host batch (dict of numpy arrays) -> Results."""
        off = np.ascontiguousarray(batch["trace_off"], dtype=np.int64)
        lat = np.ascontiguousarray(batch["lat"], dtype=np.float32)
        lon = np.ascontiguousarray(batch["lon"], dtype=np.float32)
        tm = np.ascontiguousarray(batch["time"], dtype=np.float64)
        acc = np.ascontiguousarray(batch["accuracy"], dtype=np.float32)
        b = _lib.Batch(len(off) - 1, int(off[-1]), off.ctypes.data, lat.ctypes.data, lon.ctypes.data,
                       tm.ctypes.data, acc.ctypes.data)
        r = _lib.Results()
        _check(lib().otm_match_soa(self.h, C.byref(b), C.byref(r)))
        return Results(r)

    def match_compact(self, batch):
        """Host batch -> Results through otm_match_compact: the batch narrowed
        to the Java host's own integers (compact_batch), 14 B per point over
        the link, widened on the device."""
        cb = compact_batch(batch)
        b = _lib.BatchCompact(len(cb["trace_off"]) - 1, int(cb["trace_off"][-1]), cb["trace_off"].ctypes.data,
                              cb["time_base"].ctypes.data, cb["lat"].ctypes.data, cb["lon"].ctypes.data,
                              cb["time_delta"].ctypes.data, cb["accuracy"].ctypes.data)
        r = _lib.Results()
        _check(lib().otm_match_compact(self.h, C.byref(b), C.byref(r)))
        return Results(r)

    def match_device(self, trace_off, lat, lon, time, accuracy, stream=None):
        """Device batch: torch tensors already in this GPU's HBM.  Results
        stay on the device; call fetch() for a host copy."""
        n_traces = trace_off.numel() - 1
        b = _lib.Batch(n_traces, int(lat.numel()), trace_off.data_ptr(), lat.data_ptr(), lon.data_ptr(),
                       time.data_ptr(), accuracy.data_ptr())
        _check(lib().otm_match_device(self.h, C.byref(b), C.c_void_p(stream) if stream else None))

    def fetch(self):
        r = _lib.Results()
        _check(lib().otm_fetch_results(self.h, C.byref(r)))
        return Results(r)

    def hist_bind(self, tensor, nbins, bin_kph, speed_sum=None):
        """Per-segment speed histogram (u32 counts [n_segments * nbins]) and,
        optionally, the per-segment speed sums (int64 [n_segments], 1/1000
        km/h), both caller-owned device tensors (otm_hist_bind_ex)."""
        ptr = None if tensor is None else tensor.data_ptr()
        sp = None if speed_sum is None or tensor is None else speed_sum.data_ptr()
        _check(lib().otm_hist_bind_ex(self.h, ptr, nbins, bin_kph, sp))

    def graph_info(self):
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        _check(lib().otm_graph_info(self.h, C.byref(a), C.byref(b), C.byref(c)))
        return {"nodes": a.value, "edges": b.value, "segments": c.value}

    def index_info(self):
        r, e, i, ms = C.c_float(), C.c_int64(), C.c_int32(), C.c_float()
        _check(lib().otm_index_info(self.h, C.byref(r), C.byref(e), C.byref(i), C.byref(ms)))
        return {"radius_m": r.value, "entries": e.value, "incomplete_rows": i.value, "build_ms": ms.value}

    def index_levels(self):
        """The near indexes: [{"radius_m": r, "entries": n}, ...], smallest radius first."""
        r = (C.c_float * 8)()
        e = (C.c_int64 * 8)()
        n = lib().otm_index_levels(self.h, r, e, 8)
        if n < 0:
            raise OtmError("otm_index_levels failed: %s" % _lib.last_error())
        return [{"radius_m": r[i], "entries": e[i]} for i in range(min(n, 8))]

    def index_tables(self):
        """The route index's device tables (full + near): {"slots", "bytes",
        "load_pct"} (otm_index_tables)."""
        n, b, p = C.c_int64(), C.c_int64(), C.c_int32()
        _check(lib().otm_index_tables(self.h, C.byref(n), C.byref(b), C.byref(p)))
        return {"slots": n.value, "bytes": b.value, "load_pct": p.value}

    def grid_info(self):
        cd, r, c, n, m = C.c_double(), C.c_int32(), C.c_int32(), C.c_int64(), C.c_int32()
        _check(lib().otm_grid_info(self.h, C.byref(cd), C.byref(r), C.byref(c), C.byref(n), C.byref(m)))
        return {"cell_deg": cd.value, "rows": r.value, "cols": c.value, "entries": n.value, "mult": m.value}

    def set_counting(self, on):
        _check(lib().otm_set_counting(self.h, 1 if on else 0))

    def counters(self):
        c = _lib.WorkCounters()
        _check(lib().otm_get_counters(self.h, C.byref(c)))
        return {n: getattr(c, n) for n in _lib.COUNTER_NAMES}

    def set_timing(self, on):
        _check(lib().otm_set_timing(self.h, 1 if on else 0))

    STAGES = ("columns", "candidates", "links_scan", "transitions", "viterbi", "route", "segment_bound",
              "segments_report")

    def stage_ms(self):
        ms = (C.c_float * 8)()
        _check(lib().otm_get_stage_ms(self.h, ms, 8))
        return dict(zip(self.STAGES, list(ms)))

    def kernel_ms(self):
        """Per-kernel times (ms) of the last timed match_device call, by kernel name."""
        n = 0
        while lib().otm_kernel_name(n):
            n += 1
        ms = (C.c_float * n)()
        _check(lib().otm_get_kernel_ms(self.h, ms, n))
        return {lib().otm_kernel_name(k).decode(): ms[k] for k in range(n)}

    def spill_stats(self):
        """Work units of the last batch that each fallback tier took."""
        st = _lib.SpillStats()
        _check(lib().otm_get_spill_stats(self.h, C.byref(st)))
        return {n: getattr(st, n) for n, _ in _lib.SpillStats._fields_ if n != "pad"}

    _DEBUG = {"ncand": (0, np.int32), "cand_edge": (1, np.int32), "cand_off": (2, np.float32),
              "cand_emis": (3, np.float32), "trans_off": (4, np.int64), "trans": (5, np.float32),
              "state": (6, np.int32), "col_prev": (7, np.int32), "route_dist": (8, np.float32),
              "gc": (9, np.float32), "ipos": (10, np.float32),
              # the last batch's inputs as the GPU request reader decoded them
              "in_trace_off": (11, np.int64), "in_lat": (12, np.float32), "in_lon": (13, np.float32),
              "in_time": (14, np.float64), "in_acc": (15, np.float32)}

    def debug(self, name):
        what, dt = self._DEBUG[name]
        need = C.c_size_t()
        _check(lib().otm_debug_fetch(self.h, what, None, 0, C.byref(need)))
        out = np.zeros(need.value // np.dtype(dt).itemsize, dtype=dt)
        _check(lib().otm_debug_fetch(self.h, what, out.ctypes.data, out.nbytes, None))
        return out


def report_segments(body, match_output, engine=None):
    """report() (py/reporter_service.py:110-215) over any matcher's output."""
    b = body.encode("utf-8") if isinstance(body, str) else body
    m = match_output.encode("utf-8") if isinstance(match_output, str) else match_output
    out = C.c_void_p()
    n = C.c_size_t()
    code = lib().otm_report_segments(engine.h if engine is not None else None, b, len(b), m, len(m), C.byref(out),
                                     C.byref(n))
    return code, take(out, n.value).decode("utf-8")


def encode_request(uuid, lat, lon, time, accuracy):
    """The Java batcher's request bytes (Batch.java:52-61, Point.java:39-45) as
    HttpClient.POST sends them (ISO-8859-1, HttpClient.java:26).  uuid: the
    record key, a str or its UTF-8 bytes."""
    lat = np.ascontiguousarray(lat, dtype=np.float32)
    lon = np.ascontiguousarray(lon, dtype=np.float32)
    tm = np.ascontiguousarray(time, dtype=np.int64)
    acc = np.ascontiguousarray(accuracy, dtype=np.int32)
    out = C.c_void_p()
    n = C.c_size_t()
    ub = uuid if isinstance(uuid, bytes) else uuid.encode("utf-8")
    _check(lib().otm_encode_request(ub, len(lat), lat.ctypes.data, lon.ctypes.data,
                                    tm.ctypes.data, acc.ctypes.data, C.byref(out), C.byref(n)))
    return take(out, n.value)


def murmur2_partition(key, n):
    """Kafka DefaultPartitioner shard of a uuid (Reporter.java:97 keys by uuid)."""
    b = key.encode("utf-8") if isinstance(key, str) else key
    return (lib().otm_murmur2(b, len(b)) & 0x7fffffff) % n
