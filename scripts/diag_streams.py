#!/usr/bin/env python3
"""Throughput of config 2 with 1..3 batches in flight: one engine per
in-flight batch, each on its own HIP stream, driven by its own host thread
(ctypes releases the GIL).  Prints ms per 1M-point batch for each setting."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from reporter_amd import Engine, synth
    dev = torch.device("cuda", 0)
    graph = synth.cached_graph(2)
    batch = synth.make_traces(graph, **synth.CONFIGS[2]["traces"])
    d = [torch.from_numpy(batch[k]).to(dev) for k in ("trace_off", "lat", "lon", "time", "accuracy")]
    P = int(batch["trace_off"][-1])
    engines = [Engine(graph_path=graph) for _ in range(3)]
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    steps = 24
    for e, s in zip(engines, streams):
        for _ in range(2):
            e.match_device(*d, stream=s.cuda_stream)
    torch.cuda.synchronize()
    for k in (1, 2, 3, 1, 2):
        def work(i):
            for _ in range(steps // k):
                engines[i].match_device(*d, stream=streams[i].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        th = [threading.Thread(target=work, args=(i,)) for i in range(k)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        n = (steps // k) * k
        print(json.dumps({"inflight": k, "ms_per_batch": dt * 1e3 / n, "points_per_s": P * n / dt}), flush=True)


if __name__ == "__main__":
    main()
