#!/usr/bin/env python3
"""The async JSON path (otm_submit_batch / otm_poll) at config 2's batch size:
the 10k Java request bodies submitted ROUNDS times in a row, polled until all
responses are back; points/s, with the library's own settings taken from the
environment (OTM_ASYNC_WORKERS, OTM_ASYNC_BATCH, OTM_JSON_PROFILE).  Prints
one JSON line.  A/B tooling for bench.py's json_report.async figure."""
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
    rounds = int(os.environ.get("ROUNDS", "5"))
    tr = dict(synth.CONFIGS[2]["traces"])
    b = synth.make_traces(graph, **tr)
    P = int(b["trace_off"][-1])
    nb = len(b["trace_off"]) - 1
    bodies = []
    for t in range(nb):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        bodies.append(encode_request("veh%d" % t, b["lat"][a:e], b["lon"][a:e], b["time"][a:e].astype(np.int64),
                                     b["accuracy"][a:e].astype(np.int32)))
    arr = (C.c_char_p * nb)(*bodies)
    lens = (C.c_size_t * nb)(*[len(x) for x in bodies])
    arena = None
    if os.environ.get("ARENA", "1") == "1":  # the bodies in a request arena (otm_request_arena_alloc)
        from reporter_amd import RequestArena
        arena = RequestArena(bodies)
        arr, lens = arena.ptrs, arena.lens
    tags = [(C.c_uint64 * nb)(*range(r * nb, (r + 1) * nb)) for r in range(rounds)]
    rdt = np.dtype([("tag", "<u8"), ("code", "<i4"), ("pad", "<i4"), ("body", "<u8"), ("len", "<u8")])
    cap = 1 << 16
    rbuf = (_lib.Result * cap)()
    out = {"env": {k: os.environ.get(k) for k in ("OTM_ASYNC_WORKERS", "OTM_ASYNC_BATCH", "OTM_HOST_THREADS", "ARENA")}}
    with Engine(graph_path=graph) as eng:
        def run():
            parts, got = [], 0
            t0 = time.perf_counter()
            ts = []
            for r in range(rounds):
                assert L.otm_submit_batch(eng.h, nb, arr, lens, tags[r]) == 0
                ts.append(time.perf_counter() - t0)
            while got < nb * rounds:
                n = L.otm_poll(eng.h, rbuf, cap, 200000)
                if n > 0:
                    parts.append(np.frombuffer(rbuf, dtype=rdt, count=n).copy())
                    got += n
            dt = time.perf_counter() - t0
            rr = np.concatenate(parts)
            for pb in rr["body"]:
                L.otm_free(C.c_void_p(int(pb)))
            return dt, ts
        run()
        res = []
        for _ in range(3):
            dt, ts = run()
            res.append(dt)
        best = min(res)
        out.update({"points_per_s": P * rounds / best, "points_per_s_mean": P * rounds * len(res) / sum(res), "seconds": res, "submit_returned_at_s": ts,
                    "requests": nb * rounds})
        # one call at a time, for comparison
        outs = (C.c_void_p * nb)()
        olens = (C.c_size_t * nb)()
        codes = (C.c_int * nb)()
        assert L.otm_report_batch(eng.h, nb, arr, lens, outs, olens, codes) == 0  # warm (the pipeline's contexts)
        for i in range(nb):
            L.otm_free(outs[i])
        t0 = time.perf_counter()
        for _ in range(rounds):
            assert L.otm_report_batch(eng.h, nb, arr, lens, outs, olens, codes) == 0
            for i in range(nb):
                L.otm_free(outs[i])
        out["one_call_points_per_s"] = P * rounds / (time.perf_counter() - t0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
