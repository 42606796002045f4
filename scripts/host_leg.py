#!/usr/bin/env python3
"""The host-inclusive leg alone (bench.py's host_inclusive, config 2): LEG =
compact | soa | both (alternating), three batches in flight from three host
threads, STEPS steps per run; prints one JSON line.  A/B and profiling tool."""
import ctypes as C
import itertools
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (the HIP runtime the library binds to)
    from reporter_amd import Engine, _lib, synth
    from reporter_amd.engine import compact_batch
    L = _lib.lib()
    leg = os.environ.get("LEG", "both")
    steps = int(os.environ.get("STEPS", "30"))
    inflight = int(os.environ.get("INFLIGHT", "3"))
    graph = synth.cached_graph(2)
    b = synth.make_traces(graph, **synth.CONFIGS[2]["traces"])
    P = int(b["trace_off"][-1])
    nt = len(b["trace_off"]) - 1
    pinned = []

    def bufs(arrays):
        out = {}
        for k, a in arrays.items():
            a = np.ascontiguousarray(a)
            p = L.otm_host_alloc(max(a.nbytes, 1))
            C.memmove(p, a.ctypes.data, a.nbytes)
            pinned.append(p)
            out[k] = p
        return out

    hp = bufs({k: b[k] for k in ("trace_off", "lat", "lon", "time", "accuracy")})
    hb = _lib.Batch(nt, P, hp["trace_off"], hp["lat"], hp["lon"], hp["time"], hp["accuracy"])
    cb = compact_batch(b)
    hc = bufs(cb)
    hcb = _lib.BatchCompact(nt, P, hc["trace_off"], hc["time_base"], hc["lat"], hc["lon"], hc["time_delta"],
                            hc["accuracy"])
    eng = Engine(graph_path=graph)
    engines = [eng] + [eng.clone() for _ in range(inflight - 1)]
    outs = [_lib.Results() for _ in engines]

    def soa(i):
        assert L.otm_match_soa(engines[i].h, C.byref(hb), C.byref(outs[i])) == 0

    def compact(i):
        assert L.otm_match_compact(engines[i].h, C.byref(hcb), C.byref(outs[i])) == 0

    def run(call):
        for i in range(inflight):
            call(i)
        tick = itertools.count()
        gate = threading.Barrier(inflight + 1)

        def w(i):
            gate.wait()
            while next(tick) < steps:
                call(i)

        th = [threading.Thread(target=w, args=(i,)) for i in range(inflight)]
        for t in th:
            t.start()
        t0 = time.perf_counter()
        gate.wait()
        for t in th:
            t.join()
        return (time.perf_counter() - t0) * 1e3 / steps

    res = {"soa": [], "compact": []}
    for _ in range(int(os.environ.get("ROUNDS", "3"))):
        if leg in ("soa", "both"):
            res["soa"].append(run(soa))
        if leg in ("compact", "both"):
            res["compact"].append(run(compact))
    for e in engines[1:]:
        e.close()
    eng.close()
    for p in pinned:
        L.otm_host_free(p)
    print(json.dumps({"ms_per_step": res, "points": P, "inflight": inflight}))


if __name__ == "__main__":
    main()
