#!/usr/bin/env python3
"""what one oversized trace costs its batch.

A 16k-trace batch (~1M points) on the dense 32 m test grid
(tests/test_no_limits.py dense_grid) holds, in its middle, one two-point trace
whose 600 s gap needs the huge search tier.  On a fresh engine the tier has no
tables: the batch stops at that tier, the host makes them, and the batch runs
again -- whole (OTM_NO_RESUME=1, rounds 1-5) or resumed at the tier (round 6).
Times otm_match_soa (Engine.match) per call, one batch context:
  base     the batch without the long-gap trace (engine warmed),
  resumed  a fresh (warmed) engine's first call on the batch,
  clean    the same call again (tables kept),
  whole    a fresh engine's first call with OTM_NO_RESUME=1,
with each call's spill stats (attempts, resumed), and checks the results
equal.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch  # noqa: F401  (the HIP runtime torch ships)
    from reporter_amd import Engine, synth
    from test_no_limits import GRID_MEILI, grid_batch
    g = synth.make_graph("/tmp/redo_grid32.otmg", width_m=12000, height_m=12000, block_m=32, jitter_m=0,
                         arterial_every=8, highway_every=1000, complex_every=4, seg_max_m=300)
    n = int(os.environ.get("REDO_TRACES", "16383"))
    normal = synth.make_traces(g, n, 60, interval_s=5.0, noise_sigma_m=5.0, accuracy=5.0, seed=11)
    far = grid_batch(g)
    a0 = int(far["trace_off"][0])
    far2 = {k: far[k][a0:a0 + 2] for k in ("lat", "lon", "time", "accuracy")}  # one 600 s step

    def join(parts):
        out = {k: np.concatenate([p[k] for p in parts]) for k in ("lat", "lon", "time", "accuracy")}
        lens = []
        for p in parts:
            if "trace_off" in p:
                lens.extend(np.diff(p["trace_off"]).tolist())
            else:
                lens.append(len(p["lat"]))
        out["trace_off"] = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        return out

    def sl(b, t0, t1):
        return synth.slice_batch(b, t0, t1)
    half = n // 2
    batch = join([sl(normal, 0, half), far2, sl(normal, half, n)])
    warm = sl(normal, 0, 64)

    def timed(eng, b):
        t = time.perf_counter()
        r = eng.match(b)
        dt = time.perf_counter() - t
        return dt, r, eng.spill_stats()

    def same(r1, r2):
        return all(getattr(r1, k).tobytes() == getattr(r2, k).tobytes()
                   for k in ("traces", "segments", "reports", "way_ids"))

    out = {"traces": n + 1, "points": int(batch["trace_off"][-1]),
           "long_gap_trace": "2 points 600 s apart on the 32 m grid (a huge-tier search)"}
    with Engine(graph_path=g, **GRID_MEILI) as eng:
        eng.match(warm)
        timed(eng, normal)
        out["base_s"], _, _ = timed(eng, normal)
    with Engine(graph_path=g, **GRID_MEILI) as eng:
        eng.match(warm)
        out["resumed_s"], r1, s1 = timed(eng, batch)
        out["clean_s"], r2, s2 = timed(eng, batch)
        out["clean_again_s"], _, _ = timed(eng, batch)
    os.environ["OTM_NO_RESUME"] = "1"
    with Engine(graph_path=g, **GRID_MEILI) as eng:
        eng.match(warm)
        out["whole_s"], r3, s3 = timed(eng, batch)
    out["stats"] = {k: {"attempts": v["attempts"], "resumed": v["resumed"], "trans_huge": v["trans_huge"],
                        "route_huge": v["route_huge"]} for k, v in (("resumed", s1), ("clean", s2), ("whole", s3))}
    out["results_equal"] = same(r1, r2) and same(r1, r3)
    clean = min(out["clean_s"], out["clean_again_s"])
    out["resumed_over_clean"] = out["resumed_s"] / clean
    out["whole_over_clean"] = out["whole_s"] / clean
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
