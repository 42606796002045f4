#!/usr/bin/env python3
"""Soak test on the GPU box: many request batches through one engine and one
multi-device engine (members on repeated device 0), checking every call's
responses are byte-identical to the first and that host RSS and free device
memory do not drift.  One JSON line out."""
import ctypes as C
import hashlib
import json
import os
import resource
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from reporter_amd import Engine, _lib, encode_request, synth
    L = _lib.lib()
    graph = synth.cached_graph(2)
    tr = dict(synth.CONFIGS[2]["traces"])
    nveh = int(os.environ.get("OTM_SOAK_VEH", "2000"))  # (>= 4096: otm_report_batch splits the call)
    tr["n_vehicles"] = nveh
    b = synth.make_traces(graph, **tr)
    bodies = []
    for t in range(nveh):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        bodies.append(encode_request("veh%d" % t, b["lat"][a:e], b["lon"][a:e], b["time"][a:e].astype(np.int64),
                                     b["accuracy"][a:e].astype(np.int32)))
    n = len(bodies)
    arr = (C.c_char_p * n)(*bodies)
    lens = (C.c_size_t * n)(*[len(x) for x in bodies])
    outs = (C.c_void_p * n)()
    olens = (C.c_size_t * n)()
    codes = (C.c_int * n)()
    iters = int(os.environ.get("OTM_SOAK_ITERS", "300"))
    out = {"requests_per_call": n, "iterations": iters}
    for name, devs in (("one", [0]), ("group", [0, 0])):
        with Engine(graph_path=graph, devices=devs) as eng:
            ref = None
            rss0 = free0 = None
            t0 = time.perf_counter()
            for it in range(iters):
                assert L.otm_report_batch(eng.h, n, arr, lens, outs, olens, codes) == 0
                h = hashlib.sha256()
                for i in range(n):
                    h.update(C.string_at(outs[i], olens[i]))
                    L.otm_free(outs[i])
                d = h.hexdigest()
                if ref is None:
                    ref = d
                assert d == ref, "responses changed at iteration %d" % it
                if it == 10:
                    rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
                    free0 = torch.cuda.mem_get_info(0)[0]
            out[name] = {"seconds": time.perf_counter() - t0,
                         "rss_growth_kb_after_warmup": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - rss0,
                         "device_free_drop_mb_after_warmup": (free0 - torch.cuda.mem_get_info(0)[0]) / 2**20,
                         "identical": True}
    # async submit/poll: every body submitted, polled back by tag, byte-equal
    # to the batch call's response
    with Engine(graph_path=graph) as eng:
        want = [x for x in eng.report_batch(bodies)]
        t0 = time.perf_counter()
        rss_a = None
        for rnd in range(max(1, iters // 30)):
            for k, body in enumerate(bodies):
                eng.submit(body, k)
            seen = {}
            while len(seen) < n:
                for tag, code, resp in eng.poll(4096, 2000000):
                    seen[tag] = (code, resp)
            assert [seen[k] for k in range(n)] == want
            if rnd == 2:
                rss_a = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
        out["submit_poll"] = {"rounds": max(1, iters // 30), "seconds": time.perf_counter() - t0,
                              "rss_growth_kb_after_warmup": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - (rss_a or 0)
                              if rss_a else None, "identical": True}
    # engine create / destroy cycles give their device memory back
    free_a = torch.cuda.mem_get_info(0)[0]
    for _ in range(20):
        with Engine(graph_path=graph, devices=[0, 0]) as eng:
            eng.report_batch(bodies[:50])
    torch.cuda.synchronize()
    out["create_destroy"] = {"cycles": 20, "device_free_drop_mb": (free_a - torch.cuda.mem_get_info(0)[0]) / 2**20}
    # engines whose async pipeline started (three clones with streams on
    # hardware queues of their own, and its copy stream): created, used and
    # destroyed 20 times -- the queues and device memory come back
    free_b = torch.cuda.mem_get_info(0)[0]
    m = min(n, 600)
    for _ in range(20):
        with Engine(graph_path=graph) as eng:
            eng.submit_batch(bodies[:m], list(range(m)))
            got = 0
            while got < m:
                got += len(eng.poll(4096, 2000000))
    torch.cuda.synchronize()
    out["async_create_destroy"] = {"cycles": 20, "device_free_drop_mb": (free_b - torch.cuda.mem_get_info(0)[0]) / 2**20}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
