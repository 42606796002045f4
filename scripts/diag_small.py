#!/usr/bin/env python3
"""Fixed cost of one engine round trip at the small batch sizes the batcher
produces (config 5): host SoA in -> results out (otm_match_soa), split into
match_device (inputs already in HBM, one sync) and fetch, and the kernel sum."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from reporter_amd import Engine, _lib, synth
    from reporter_amd._lib import lib
    graph = synth.cached_graph(2)
    full = synth.make_traces(graph, **synth.CONFIGS[2]["traces"])
    out = []
    with Engine(graph_path=graph) as eng:
        for nt, npt in [(100, 2), (1000, 2), (10000, 2), (10000, 5), (10000, 20), (10000, 100)]:
            # first npt points of the first nt vehicles
            idx = np.concatenate([np.arange(full["trace_off"][v], full["trace_off"][v] + npt) for v in range(nt)])
            off = np.arange(nt + 1, dtype=np.int64) * npt
            lat = np.ascontiguousarray(full["lat"][idx], np.float32)
            lon = np.ascontiguousarray(full["lon"][idx], np.float32)
            tm = np.ascontiguousarray(full["time"][idx], np.float64)
            acc = np.ascontiguousarray(full["accuracy"][idx], np.float32)
            b = _lib.Batch(nt, len(idx), off.ctypes.data, lat.ctypes.data, lon.ctypes.data, tm.ctypes.data,
                           acc.ctypes.data)
            r = _lib.Results()
            for _ in range(3):
                lib().otm_match_soa(eng.h, C.byref(b), C.byref(r))
            reps = 20
            t0 = time.perf_counter()
            for _ in range(reps):
                lib().otm_match_soa(eng.h, C.byref(b), C.byref(r))
            soa = (time.perf_counter() - t0) / reps * 1e3
            d = [torch.from_numpy(x).cuda() for x in (off, lat, lon, tm, acc)]
            torch.cuda.synchronize()
            tm_dev = tf = 0.0
            for _ in range(reps):
                t0 = time.perf_counter()
                eng.match_device(*d)
                t1 = time.perf_counter()
                lib().otm_fetch_results(eng.h, C.byref(r))
                t2 = time.perf_counter()
                tm_dev += t1 - t0
                tf += t2 - t1
            eng.set_timing(True)
            eng.match_device(*d)
            km = eng.kernel_ms()
            ks = float(sum(km.values()) if isinstance(km, dict) else sum(km))
            eng.set_timing(False)
            line = {"small_points": os.environ.get("OTM_SMALL_POINTS", "default"), "traces": nt, "pts": npt, "soa_ms": round(soa, 3), "match_device_ms": round(tm_dev / reps * 1e3, 3),
                    "fetch_ms": round(tf / reps * 1e3, 3), "kernel_sum_ms": round(ks, 3),
                    "kernels_us": {k: round(v * 1e3, 1) for k, v in km.items() if v > 0}}
            print(json.dumps(line), flush=True)
            out.append(line)


if __name__ == "__main__":
    main()
