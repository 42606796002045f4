"""ctypes binding of libotmatch.so (include/otmatch.h).

The library is built in-tree (reporter_amd/lib/libotmatch.so) by
__graft_entry__.build() / `make -C reporter_amd/csrc`.  There is no fallback:
if the library is missing, loading raises.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# OTM_LIB selects another in-tree build of the same library (A/B of compile-time variants)
LIB_PATH = os.environ.get("OTM_LIB") or os.path.join(_HERE, "lib", "libotmatch.so")

OTM_OK = 0

# ---------------------------------------------------------------- structs


class Batch(C.Structure):
    _fields_ = [("n_traces", C.c_int32), ("n_points", C.c_int64), ("trace_off", C.c_void_p), ("lat", C.c_void_p),
                ("lon", C.c_void_p), ("time", C.c_void_p), ("accuracy", C.c_void_p)]


class BatchCompact(C.Structure):
    """otm_batch_compact: int64 time bases per trace, int32 time deltas and
    int16 accuracies per point (include/otmatch.h)."""
    _fields_ = [("n_traces", C.c_int32), ("n_points", C.c_int64), ("trace_off", C.c_void_p),
                ("time_base", C.c_void_p), ("lat", C.c_void_p), ("lon", C.c_void_p), ("time_delta", C.c_void_p),
                ("accuracy", C.c_void_p)]


class Results(C.Structure):
    _fields_ = [("n_traces", C.c_int32), ("n_segments", C.c_int32), ("n_reports", C.c_int32),
                ("n_way_ids", C.c_int32), ("traces", C.c_void_p), ("segments", C.c_void_p), ("reports", C.c_void_p),
                ("way_ids", C.c_void_p)]


class Result(C.Structure):
    _fields_ = [("tag", C.c_uint64), ("code", C.c_int), ("body", C.c_void_p), ("body_len", C.c_size_t)]


COUNTER_NAMES = ("points", "columns", "cells_visited", "cell_entries_scanned", "candidates", "searches", "nodes_settled",
                 "edges_relaxed", "transitions", "route_searches", "route_nodes_settled", "route_edges_relaxed",
                 "route_edges", "segments_out", "reports_out")


class WorkCounters(C.Structure):
    _fields_ = [(n, C.c_int64) for n in COUNTER_NAMES]


class SpillStats(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("cand_wave", "trans_online", "trans_wave", "trans_global", "route_online",
                                         "route_wave", "route_global", "cand_big", "trans_huge", "route_huge",
                                         "attempts", "resumed")]


class BatcherCfg(C.Structure):
    _fields_ = [("report_dist", C.c_int32), ("report_count", C.c_int32), ("report_time_s", C.c_int64),
                ("session_gap_ms", C.c_int64), ("max_batch", C.c_int32), ("json_path", C.c_int32),
                ("max_pending", C.c_int64), ("threads", C.c_int32), ("reserved", C.c_int32)]


class Forward(C.Structure):
    _fields_ = [("key", C.c_void_p), ("key_len", C.c_size_t), ("body", C.c_void_p), ("body_len", C.c_size_t),
                ("seq", C.c_int64)]


BATCHER_STATS = ("records", "clean_ops", "close_ops", "requests", "request_points", "match_batches", "forwarded",
                 "null_batch_in_clean", "keys", "stored_batches", "stored_points", "us_enqueue", "us_run",
                 "us_prepare", "us_match", "us_apply", "raw_messages", "raw_dropped", "us_format", "null_responses")


class BatcherStats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in BATCHER_STATS]


class Formatted(C.Structure):
    _fields_ = [("n", C.c_int32), ("n_ok", C.c_int32), ("ok", C.c_void_p), ("key_off", C.c_void_p),
                ("keys", C.c_void_p), ("lat", C.c_void_p), ("lon", C.c_void_p), ("accuracy", C.c_void_p),
                ("time", C.c_void_p)]


# int (*otm_report_fn)(void* ctx, int n, const char* const* reqs, const size_t* lens, char** resps,
#                      size_t* resp_lens, int* codes)
REPORT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t),
                        C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_int))


class SynthGraphParams(C.Structure):
    _fields_ = [("center_lat", C.c_double), ("center_lon", C.c_double), ("width_m", C.c_double),
                ("height_m", C.c_double), ("block_m", C.c_double), ("jitter_m", C.c_double),
                ("arterial_every", C.c_int), ("highway_every", C.c_int), ("unassoc_frac", C.c_double),
                ("complex_every", C.c_int), ("seg_max_m", C.c_double), ("cell_deg", C.c_double),
                ("seed", C.c_uint64)]


class MeiliParams(C.Structure):
    """otm_meili_params (include/otmatch.h)"""
    _fields_ = [(n, C.c_float) for n in ("sigma_z", "beta", "max_route_distance_factor", "breakage_distance",
                                         "interpolation_distance", "search_radius", "max_search_radius",
                                         "gps_accuracy", "turn_penalty_factor")] + [("max_candidates", C.c_int32)]


class SynthTraceParams(C.Structure):
    _fields_ = [("n_vehicles", C.c_int32), ("points_per_vehicle", C.c_int32), ("interval_s", C.c_double),
                ("noise_sigma_m", C.c_double), ("accuracy", C.c_float), ("t0", C.c_double), ("seed", C.c_uint64),
                ("vehicle_offset", C.c_int32), ("vehicle_ids", C.c_void_p)]


SEGMENT_DTYPE = np.dtype([("segment_id", "<i8"), ("start_time", "<f8"), ("end_time", "<f8"), ("length", "<i4"),
                          ("queue_length", "<i4"), ("begin_shape_index", "<i4"), ("end_shape_index", "<i4"),
                          ("way_off", "<i4"), ("way_cnt", "<i4"), ("flags", "<u4"), ("pad", "<u4")])
REPORT_DTYPE = np.dtype([("id", "<i8"), ("next_id", "<i8"), ("t0", "<f8"), ("t1", "<f8"), ("length", "<i4"),
                         ("queue_length", "<i4"), ("flags", "<u4"), ("pad", "<u4")])
TRACE_DTYPE = np.dtype([(n, "<i4") for n in (
    "code", "error_kind", "seg_off", "seg_cnt", "rep_off", "rep_cnt", "shape_used", "successful_count",
    "unreported_count", "discontinuities", "invalid_speeds", "unassociated", "successful_length",
    "unreported_length")])

SEG_START_VALID, SEG_END_VALID, SEG_INTERNAL, SEG_START_INT, SEG_END_INT = 1, 2, 4, 8, 16
REP_T1_INT, REP_T0_INT = 1, 2
REP_T1_INT_MINUS1 = REP_T1_INT

_lib = None


def _declare(L):
    vp, sz, i32, i64 = C.c_void_p, C.c_size_t, C.c_int32, C.c_int64
    pp = C.POINTER(C.c_void_p)
    psz = C.POINTER(C.c_size_t)
    sig = {
        "otm_engine_create": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.c_int, pp]),
        "otm_engine_members": (C.c_int, [vp]),
        "otm_config_meili": (C.c_int, [C.c_char_p, vp]),
        "otm_request_points": (C.c_int, [C.c_char_p, sz, C.c_int, vp, vp, vp, vp, C.c_int, C.c_char_p, sz]),
        "otm_engine_member": (vp, [vp, C.c_int]),
        "otm_engine_destroy": (None, [vp]),
        "otm_last_error": (C.c_char_p, [vp]),
        "otm_free": (None, [vp]),
        "otm_report": (C.c_int, [vp, C.c_char_p, sz, pp, psz]),
        "otm_report_batch": (C.c_int, [vp, C.c_int, C.POINTER(C.c_char_p), psz, pp, psz, C.POINTER(C.c_int)]),
        "otm_match_json": (C.c_int, [vp, C.c_char_p, sz, pp, psz]),
        "otm_report_segments": (C.c_int, [vp, C.c_char_p, sz, C.c_char_p, sz, pp, psz]),
        "otm_submit": (C.c_int, [vp, C.c_char_p, sz, C.c_uint64]),
        "otm_poll": (C.c_int, [vp, C.POINTER(Result), C.c_int, C.c_int]),
        "otm_submit_batch": (C.c_int, [vp, C.c_int, vp, vp, vp]),
        "otm_encode_request": (C.c_int, [C.c_char_p, C.c_int, vp, vp, vp, vp, pp, psz]),
        "otm_match_soa": (C.c_int, [vp, C.POINTER(Batch), C.POINTER(Results)]),
        "otm_match_compact": (C.c_int, [vp, C.POINTER(BatchCompact), C.POINTER(Results)]),
        "otm_request_arena_alloc": (vp, [sz]),
        "otm_request_arena_release": (C.c_int, [vp]),
        "otm_host_alloc": (vp, [sz]),
        "otm_host_free": (None, [vp]),
        "otm_match_device": (C.c_int, [vp, C.POINTER(Batch), vp]),
        "otm_fetch_results": (C.c_int, [vp, C.POINTER(Results)]),
        "otm_hist_bind": (C.c_int, [vp, vp, C.c_int, C.c_float]),
        "otm_hist_bind_ex": (C.c_int, [vp, vp, C.c_int, C.c_float, vp]),
        "otm_report_segments_device": (C.c_int, [vp, C.c_int, C.POINTER(C.c_char_p), psz, C.POINTER(C.c_char_p), psz,
                                                 pp, psz, C.POINTER(C.c_int)]),
        "otm_graph_info": (C.c_int, [vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]),
        "otm_index_info": (C.c_int, [vp, C.POINTER(C.c_float), C.POINTER(i64), C.POINTER(i32),
                                     C.POINTER(C.c_float)]),
        "otm_index_levels": (C.c_int, [vp, C.POINTER(C.c_float), C.POINTER(i64), C.c_int]),
        "otm_index_tables": (C.c_int, [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
        "otm_grid_info": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(i32), C.POINTER(i32), C.POINTER(i64),
                                    C.POINTER(i32)]),
        "otm_set_counting": (C.c_int, [vp, C.c_int]),
        "otm_get_counters": (C.c_int, [vp, C.POINTER(WorkCounters)]),
        "otm_set_timing": (C.c_int, [vp, C.c_int]),
        "otm_get_stage_ms": (C.c_int, [vp, C.POINTER(C.c_float), C.c_int]),
        "otm_get_kernel_ms": (C.c_int, [vp, C.POINTER(C.c_float), C.c_int]),
        "otm_kernel_name": (C.c_char_p, [C.c_int]),
        "otm_get_spill_stats": (C.c_int, [vp, C.POINTER(SpillStats)]),
        "otm_debug_fetch": (C.c_int, [vp, C.c_int, vp, sz, psz]),
        "otm_kmax": (C.c_int, []),
        "otm_debug_py_repr": (C.c_int, [C.c_double, C.c_char_p]),
        "otm_debug_py_round3": (C.c_int, [C.c_double, C.POINTER(C.c_double)]),
        "otm_debug_arena_stress": (C.c_int, [C.c_int, C.c_int]),
        "otm_debug_last_split": (C.c_int, [vp]),
        "otm_batcher_defaults": (None, [C.POINTER(BatcherCfg)]),
        "otm_batcher_create": (C.c_int, [vp, C.POINTER(BatcherCfg), REPORT_FN, vp, pp]),
        "otm_batcher_destroy": (None, [vp]),
        "otm_batcher_process": (C.c_int, [vp, C.c_int, C.POINTER(C.c_char_p), psz, vp, vp, vp, vp, vp]),
        "otm_batcher_flush": (C.c_int, [vp]),
        "otm_batcher_close": (C.c_int, [vp]),
        "otm_batcher_take": (C.c_int, [vp, C.POINTER(Forward), C.c_int]),
        "otm_batcher_get_stats": (C.c_int, [vp, C.POINTER(BatcherStats)]),
        "otm_batcher_batch": (C.c_int, [vp, C.c_char_p, sz, C.c_int, vp, vp, vp, vp, C.POINTER(C.c_float)]),
        "otm_quantize_decimal6": (None, [vp, vp, C.c_int64]),
        "otm_engine_clone": (C.c_int, [vp, C.POINTER(vp)]),
        "otm_formatter_create": (C.c_int, [C.c_char_p, C.POINTER(vp), C.c_char_p, sz]),
        "otm_formatter_destroy": (None, [vp]),
        "otm_format": (C.c_int, [vp, C.c_int32, vp, vp, C.c_int, C.POINTER(Formatted)]),
        "otm_formatted_free": (None, [C.POINTER(Formatted)]),
        "otm_batcher_process_raw": (C.c_int, [vp, vp, C.c_int32, vp, vp, vp, C.c_int]),
        "otm_synth_graph_defaults": (None, [C.POINTER(SynthGraphParams)]),
        "otm_synth_graph": (C.c_int, [C.POINTER(SynthGraphParams), C.c_char_p]),
        "otm_synth_traces": (C.c_int, [C.c_char_p, C.POINTER(SynthTraceParams), vp, vp, vp, vp, vp, vp, vp]),
        "otm_murmur2": (i32, [C.c_char_p, sz]),
        "otm_synth_true_paths": (i64, [C.c_char_p, C.POINTER(SynthTraceParams), vp, vp, i64]),
        "otm_synth_true_paths_timed": (i64, [C.c_char_p, C.POINTER(SynthTraceParams), vp, vp, vp, i64]),
        "otm_tile_id": (i64, [C.c_int, C.c_double, C.c_double]),
        "otm_tile_file": (C.c_int, [i64, C.c_int, C.c_char_p, C.c_char_p, sz]),
        "otm_tile_files_bbox": (C.c_int, [C.c_double, C.c_double, C.c_double, C.c_double, C.c_char_p, pp, psz]),
        "otm_runtime_info": (C.c_char_p, []),
        "otm_stream_create": (vp, [vp, C.c_int]),
        "otm_stream_destroy": (None, [vp]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("OTM_LIB") and not hasattr(L, name):
            continue  # (an A/B build of an earlier library: its own entry points only)
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return sig


EXPORTED = None


def _bind_torch_hip_runtime():
    """Load torch's HIP runtime first when torch is present.

    torch ships its own libamdhip64 (SONAME libamdhip64.so.7, the same soname
    libotmatch.so links against).  With torch loaded first the dynamic linker
    binds libotmatch to that same runtime, so device pointers and streams are
    shared with torch (tensors, RCCL); two HIP runtimes in one process would
    each try to own the GPU.
    """
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    """The loaded library; raises if it was not built (no CPU fallback)."""
    global _lib, EXPORTED
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libotmatch.so not built (%s); run __graft_entry__.build() or "
                               "`make -C reporter_amd/csrc`" % LIB_PATH)
        _bind_torch_hip_runtime()
        L = C.CDLL(LIB_PATH)
        EXPORTED = sorted(_declare(L).keys())
        _lib = L
    return _lib


def malloc_bytes(b):
    """A malloc'd copy of `b` (for bodies handed to the library, released by otm_free)."""
    libc = C.CDLL(None)
    libc.malloc.restype = C.c_void_p
    libc.malloc.argtypes = [C.c_size_t]
    p = libc.malloc(len(b) + 1)
    C.memmove(p, b + b"\0", len(b) + 1)
    return p


def last_error():
    msg = lib().otm_last_error(None)
    return msg.decode("utf-8", "replace") if msg else ""


def take(ptr, n):
    """Copy a library-allocated buffer into bytes and free it."""
    s = C.string_at(ptr, n)
    lib().otm_free(ptr)
    return s


def as_array(ptr, dtype, n):
    if not n or not ptr:
        return np.zeros(0, dtype=dtype)
    nbytes = n * np.dtype(dtype).itemsize
    buf = (C.c_char * nbytes).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=n).copy()


def runtime_info():
    """Path of the HIP runtime libotmatch is bound to, and its version."""
    return lib().otm_runtime_info().decode()
