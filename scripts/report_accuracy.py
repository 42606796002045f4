#!/usr/bin/env python3
"""Datastore-report accuracy of a config against the synthetic ground truth
(DESIGN.md §3.2), on the CPU oracle (the GPU path is bit-identical to it):
synth.report_agreement over the whole batch, and how many interior report
errors sit in traces with an outlier column (a probe farther from its road
than the search radius).  Prints one JSON line.

  python scripts/report_accuracy.py --config 2 [--vehicles N] [--radius R]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from oracle import pyoracle
    from reporter_amd import synth
    from reporter_amd.engine import report_segments
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2, choices=(2, 4))
    ap.add_argument("--vehicles", type=int, default=0)
    ap.add_argument("--radius", type=float, default=0.0, help="search radius (0: the config's)")
    a = ap.parse_args()
    cfg = synth.CONFIGS[a.config]
    g = synth.cached_graph(a.config)
    tp = dict(cfg["traces"])
    nv = a.vehicles or tp.pop("n_vehicles")
    tp.pop("n_vehicles", None)
    ppv = tp.pop("points_per_vehicle")
    meili = dict(cfg.get("meili", {}))
    if a.radius > 0:
        meili.update(search_radius=a.radius, max_search_radius=max(a.radius, meili.get("max_search_radius", 100.0)))
    b = synth.make_traces(g, nv, ppv, **tp)
    off, edges, enter = synth.true_paths_timed(g, nv, ppv, **tp)
    orc = pyoracle.match_batch(pyoracle.Graph(g), b, p=pyoracle.params(**meili), nthreads=os.cpu_count() or 4,
                               keep_stages=True)
    r = synth.report_agreement(g, off, edges, enter, b["trace_off"], b["time"], orc)
    # interior report errors per trace, against the traces' outlier columns
    outl = synth.outlier_points(g, b["true_edge"], orc["ncand"], orc["cand_edge"], orc["cand_off"], b["trace_off"],
                                orc["gc"])
    truth = synth.true_segments(g, off, edges, enter, None)
    tr, reps = orc["traces"], orc["reports"]
    n_int = n_int_out = 0
    for t in range(len(tr)):
        ts = b["time"][b["trace_off"][t + 1] - 1]
        ts = int(ts) if ts == int(ts) else repr(float(ts))
        body = ('{"uuid":"x","trace":[{"lat":0,"lon":0,"time":%s,"accuracy":5},{"lat":0,"lon":0,"time":%s,'
                '"accuracy":5}]}' % (ts, ts))
        code, resp = report_segments(body, json.dumps({"segments": truth[t]}, separators=(",", ":")))
        want = json.loads(resp).get("datastore", {}).get("reports", []) if code == 200 else []
        ra, rn = int(tr["rep_off"][t]), int(tr["rep_cnt"][t])
        got = reps[ra:ra + rn]
        kw = [(int(x["id"]), int(x.get("next_id", -1))) for x in want]
        kg = [(int(x), int(y)) for x, y in zip(got["id"].tolist(), got["next_id"].tolist())]
        pairs = synth._lcs_pairs(kw, kg)
        e = sum((qa - pa - 1) + (qb - pb - 1) for (pa, pb), (qa, qb) in zip(pairs, pairs[1:]))
        if e:
            n_int += e
            if outl[int(b["trace_off"][t]):int(b["trace_off"][t + 1])].any():
                n_int_out += e
    r.update(config=a.config, vehicles=nv, search_radius=meili.get("search_radius", 50.0),
             interior_errors=n_int, interior_errors_in_traces_with_outlier_columns=n_int_out,
             outlier_columns=int(np.asarray(outl).sum()))
    print(json.dumps(r))


if __name__ == "__main__":
    main()
