#!/usr/bin/env python3
"""The JSON /report path at config 2's batch size: 10k request bodies (the
Java batcher's bytes, Batch.java:52-61) through otm_report_batch in one call,
timed in C (ctypes, GIL released), against otm_match_soa on the same points.
Prints one JSON line: requests/s, points/s and ms per call for both."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from reporter_amd import Engine, _lib, encode_request, synth
    L = _lib.lib()
    graph = synth.cached_graph(2)
    n_veh = int(os.environ.get("OTM_JSON_VEH", "10000"))
    tr = dict(synth.CONFIGS[2]["traces"])
    tr["n_vehicles"] = n_veh
    b = synth.make_traces(graph, **tr)
    P = int(b["trace_off"][-1])
    bodies = []
    for t in range(n_veh):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        bodies.append(encode_request("veh%d" % t, b["lat"][a:e], b["lon"][a:e], b["time"][a:e].astype(np.int64),
                                     b["accuracy"][a:e].astype(np.int32)))
    n = len(bodies)
    arr = (C.c_char_p * n)(*bodies)
    lens = (C.c_size_t * n)(*[len(x) for x in bodies])
    outs = (C.c_void_p * n)()
    olens = (C.c_size_t * n)()
    codes = (C.c_int * n)()
    out = {"requests": n, "points": P, "request_bytes": int(sum(len(x) for x in bodies))}
    with Engine(graph_path=graph) as eng:
        def json_call():
            rc = L.otm_report_batch(eng.h, n, arr, lens, outs, olens, codes)
            assert rc == 0
            for i in range(n):
                L.otm_free(outs[i])
        for _ in range(2):
            json_call()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            json_call()
        dt = (time.perf_counter() - t0) / reps
        out["json_ms_per_call"] = dt * 1e3
        out["json_points_per_s"] = P / dt
        out["json_requests_per_s"] = n / dt
        out["response_bytes"] = int(sum(olens[i] for i in range(n)))
        assert all(codes[i] == 200 for i in range(n))
        for _ in range(2):
            eng.match(b)
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.match(b)
        dt = (time.perf_counter() - t0) / reps
        out["soa_ms_per_call"] = dt * 1e3
        out["soa_points_per_s"] = P / dt
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
