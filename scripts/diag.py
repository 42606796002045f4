#!/usr/bin/env python3
"""Per-kernel times and fallback-tier work of one config-2 batch (diagnostic)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from reporter_amd import Engine, synth
    cfg = dict(synth.CONFIGS[2]["traces"])
    nveh = int(os.environ.get("OTM_DIAG_VEHICLES", "10000"))
    cfg["n_vehicles"] = nveh
    graph = synth.cached_graph(2)
    b = synth.make_traces(graph, vehicle_ids=synth.shard_vehicle_ids(nveh, 0, 1),
                          **cfg)
    dev = torch.device("cuda", 0)
    d = {k: torch.from_numpy(b[k]).to(dev) for k in ("trace_off", "lat", "lon", "time", "accuracy")}
    radius = os.environ.get("OTM_INDEX_RADIUS")
    with Engine(graph_path=graph, index_radius_m=float(radius) if radius else None) as eng:
        info = eng.index_info()
        for _ in range(3):
            eng.match_device(d["trace_off"], d["lat"], d["lon"], d["time"], d["accuracy"])
        torch.cuda.synchronize()
        eng.set_timing(True)
        eng.match_device(d["trace_off"], d["lat"], d["lon"], d["time"], d["accuracy"])
        torch.cuda.synchronize()
        out = {"index": info, "spill": eng.spill_stats(), "kernel_ms": eng.kernel_ms(), "stage_ms": eng.stage_ms()}
        gc = eng.debug("gc")[:len(b["lat"])]
        cp = eng.debug("col_prev")[:len(b["lat"])]
        lk = cp >= 0
        out["linked_columns"] = int(lk.sum())
        out["bound_over_radius"] = int((5 * gc[lk] > info["radius_m"]).sum())
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
