#!/usr/bin/env python3
"""BASELINE config 5: the reference's batcher feeding the GPU matcher.

The config-2 fleet (10k vehicles x 100 points, 5 s sampling) becomes one
interleaved record stream ordered by record time -- what the `formatted`
topic carries -- and goes through the native batcher (BatchingProcessor +
Batch semantics, reporter_amd/csrc/batcher.cpp) with the engine as matcher.
Reports sustained records/s (ingest) and matched points/s (sum of request
trace lengths), with the request mix the reference's gates and its clean()
quirk produce.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vehicles", type=int, default=10000)
    ap.add_argument("--points", type=int, default=100)
    ap.add_argument("--chunk", type=int, default=20000, help="records per otm_batcher_process call (one poll)")
    ap.add_argument("--json-path", action="store_true")
    ap.add_argument("--max-pending", type=int, default=100000, help="queued operations that trigger a drain")
    ap.add_argument("--raw", choices=["json", "sv"], default=None,
                    help="feed raw messages through the native formatter (README's json / sv layouts)")
    ap.add_argument("--format-threads", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8, help="batcher host threads (otm_batcher_cfg.threads)")
    ap.add_argument("--cpu-sample", type=int, default=100000,
                    help="records of the same stream for the CPU baseline (0: skip)")
    args = ap.parse_args()
    import torch  # noqa: F401  (binds the HIP runtime torch ships)
    from reporter_amd import Engine, synth
    from reporter_amd.batcher import Batcher, KeyBlock
    graph = synth.cached_graph(2)
    tr = dict(synth.CONFIGS[2]["traces"], n_vehicles=args.vehicles, points_per_vehicle=args.points)
    b = synth.make_traces(graph, **tr)
    nv, npt = args.vehicles, args.points
    veh = np.repeat(np.arange(nv), npt)
    t = b["time"].astype(np.int64) + (veh % 5)  # stagger the fleet a little
    order = np.lexsort((veh, t))
    keys = np.array(["veh%d" % v for v in range(nv)], dtype=object)[veh[order]]
    lat, lon = b["lat"][order], b["lon"][order]
    acc = np.ceil(b["accuracy"][order]).astype(np.int32)
    tm = t[order]
    ts = tm * 1000
    with Engine(graph_path=graph) as eng:
        bt = Batcher(engine=eng, json_path=args.json_path, max_pending=args.max_pending, threads=args.threads)
        # warm the engine (allocations, code objects) outside the timed region
        eng.match(synth.slice_batch(b, 0, min(100, nv)))
        n = len(keys)
        if args.raw:
            from reporter_amd.formatter import Formatter, pack_messages
            if args.raw == "json":
                spec = ",json,id,latitude,longitude,timestamp,accuracy"
                msgs = ['{"timestamp":%d,"id":"%s","accuracy":%d,"latitude":%r,"longitude":%r}'
                        % (tm[i], keys[i], acc[i], float(lat[i]), float(lon[i])) for i in range(n)]
            else:
                import datetime
                spec = ",sv,\\|,1,9,10,0,5,yyyy-MM-dd HH:mm:ss"
                ep = datetime.datetime(1970, 1, 1)
                msgs = ["%s|%s|x|x|x|%d|x|x|x|%r|%r|x|x|x"
                        % ((ep + datetime.timedelta(seconds=int(tm[i]))).strftime("%Y-%m-%d %H:%M:%S"), keys[i],
                           acc[i], float(lat[i]), float(lon[i])) for i in range(n)]
            fmt = Formatter(spec)
            blocks = [(i, min(n, i + args.chunk), pack_messages(msgs[i:min(n, i + args.chunk)]))
                      for i in range(0, n, args.chunk)]
            from reporter_amd._lib import lib
            t0 = time.perf_counter()
            for i, j, (buf, off) in blocks:
                tsb = np.ascontiguousarray(ts[i:j])
                rc = lib().otm_batcher_process_raw(bt.h, fmt.h, j - i, buf.ctypes.data, off.ctypes.data,
                                                   tsb.ctypes.data, args.format_threads)
                assert rc == 0, rc
        else:
            blocks = [(i, min(n, i + args.chunk), KeyBlock(list(keys[i:min(n, i + args.chunk)])))
                      for i in range(0, n, args.chunk)]
            t0 = time.perf_counter()
            for i, j, kb in blocks:
                bt.process(kb, lat[i:j], lon[i:j], acc[i:j], tm[i:j], ts[i:j])
        bt.flush()
        bt.close()
        dt = time.perf_counter() - t0
        st = bt.stats()
        fwd = len(bt.forwarded())
    cpu = None
    if args.cpu_sample > 0:
        # CPU baseline: the reference's topology restated record at a time
        # (oracle/pybatcher.py) with a synchronous /report per request into the
        # C oracle's handler -- what one Kafka Streams thread does
        sys.path.insert(0, ROOT)
        from oracle import pybatcher, pyoracle
        g = pyoracle.Graph(graph)
        bp = pybatcher.BatchingProcessor(lambda body: pyoracle.handle_request(g, body)[1])
        m = min(args.cpu_sample, n)
        tc = time.perf_counter()
        for i in range(m):
            bp.process(keys[i], pybatcher.Point(lat[i], lon[i], acc[i], tm[i]), int(ts[i]))
        dtc = time.perf_counter() - tc
        cpu = {"value": m / dtc, "unit": "records/s", "cores": 1, "kind": "port",
               "sample": "first %d records of the same stream: Python restatement of BatchingProcessor + the C "
                         "oracle's /report handler per request, one thread (one Kafka Streams thread)" % m,
               "requests": bp.requests}
    line = {"metric": "config5 sustained ingest through the native batcher + GPU matcher",
            "records_per_s": n / dt, "matched_points_per_s": st["request_points"] / dt, "seconds": dt,
            "records": n, "forwarded": fwd, "path": "json" if args.json_path else "binary",
            "batcher_threads": args.threads,
            "input": "raw %s messages via the native formatter (%d threads)" % (args.raw, args.format_threads)
            if args.raw else "formatted records", "stats": st, "cpu_baseline": cpu,
            "workload": "config-2 fleet (%d vehicles x %d points, 5 s) as one time-ordered stream" % (nv, npt)}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
