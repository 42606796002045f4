#!/usr/bin/env python3
"""Where the matched OSMLR segment sequences differ from the routes the
synthetic vehicles drove (VERDICT r3 "next" #2), on the CPU oracle.

Per trace: the segment ids of the vehicle's true edge path against the
matched ones, aligned and classified by reporter_amd.synth.classify_sequences
(start / end partial segments; interior: dropped, inserted over a probe
outside its road's search radius, U-turn excursions, other insertions,
reversed, swapped).  Per HMM column (a point that is not interpolated):
whether its matched position is the true edge, a node of it, its reverse,
another edge of the same segment, or elsewhere, split into the first / last 3
columns of a trace and the rest; and how many points had no candidate on
their true road (outliers: the probe fell outside the search radius).

    python scripts/accuracy_breakdown.py --config 2 --vehicles 2000 [--out f.json]

Writes a JSON summary (stdout, or --out).  Test infrastructure: it runs the
oracle (oracle/pyoracle.py) as the matcher it measures (the GPU path is
bit-identical to it).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from reporter_amd import synth  # noqa: E402
from oracle import pyoracle  # noqa: E402

KMAX = 32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--vehicles", type=int, default=2000)
    ap.add_argument("--points", type=int, default=100)
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--cache", default=os.environ.get("OTM_GRAPH_CACHE", "/tmp/otm_graphs"))
    ap.add_argument("--meili", default="", help="k=v,... overrides of the matcher parameters")
    ap.add_argument("--out")
    a = ap.parse_args()
    cfg = synth.CONFIGS[a.config]
    gpath = synth.cached_graph(a.config, a.cache)
    e_from = synth._graph_section(gpath, 3, np.int32)
    e_to = synth._graph_section(gpath, 4, np.int32)
    e_seg = synth._graph_section(gpath, 8, np.int32)
    e_opp = synth._graph_section(gpath, 13, np.int32)
    tr = dict(cfg["traces"])
    tr["n_vehicles"] = a.vehicles
    tr["points_per_vehicle"] = a.points
    b = synth.make_traces(gpath, **tr)
    meili = dict(cfg.get("meili", {}))
    for kv in filter(None, a.meili.split(",")):
        k, v = kv.split("=")
        meili[k] = float(v)
    t0 = time.time()
    orc = pyoracle.match_batch(pyoracle.Graph(gpath), b, p=pyoracle.params(**meili), nthreads=a.threads,
                               keep_stages=True)
    t_match = time.time() - t0
    poff, pedges = synth.true_paths(gpath, **tr)
    outlier = synth.outlier_points(gpath, b["true_edge"], orc["ncand"], orc["cand_edge"], orc["cand_off"],
                                   b["trace_off"], orc["gc"])
    per = []
    agr = synth.segment_agreement(gpath, poff, pedges, orc, trace_off=b["trace_off"], outlier=outlier, per_trace=per)
    # per column: the matched position against the true one
    state = orc["state"]
    cedge, coff = orc["cand_edge"], orc["cand_off"]
    true_edge = b["true_edge"]
    off = b["trace_off"]
    col = {}
    for t in range(a.vehicles):
        # columns (rule 1): the trace's first point and every point with gc > 0
        idx = [i for i in range(int(off[t]), int(off[t + 1])) if (i == off[t] or orc["gc"][i] > 0)]
        for r, i in enumerate(idx):
            where = "first3" if r < 3 else ("last3" if r >= len(idx) - 3 else "interior")
            s = int(state[i])
            te = int(true_edge[i])
            if s < 0:
                kind = "unmatched"
            else:
                me = int(cedge[i * KMAX + s])
                if coff[i * KMAX + s] == 0.0:  # a node candidate (carried on an out-edge of the node)
                    kind = "node_of_true_edge" if e_from[me] in (e_from[te], e_to[te]) else "other_node"
                elif me == te:
                    kind = "true_edge"
                elif me == e_opp[te]:
                    kind = "reverse_edge"
                elif e_seg[me] >= 0 and e_seg[me] == e_seg[te]:
                    kind = "same_segment"
                else:
                    kind = "other_edge"
            if outlier[i]:
                kind += "@outlier"
            d = col.setdefault(where, {})
            d[kind] = d.get(kind, 0) + 1
    # the trace ends: is the true first / last position within the search
    # radius of a node of its edge?  Among all traces and among those with a
    # start / end error.
    e_len = synth._graph_section(gpath, 5, np.float32)
    radius = float(meili.get("search_radius", 50.0))
    ends = {}
    for t in range(a.vehicles):
        c = per[t]
        for side, i in (("start", int(off[t])), ("end", int(off[t + 1]) - 1)):
            te = int(true_edge[i])
            d = min(float(b["true_off"][i]), float(e_len[te]) - float(b["true_off"][i]))
            err = c[side + "_missed"] + c[side + "_extra"] > 0
            for grp in ("all", "with_error") if err else ("all",):
                k = "%s_%s" % (side, grp)
                n, near = ends.get(k, (0, 0))
                ends[k] = (n + 1, near + (1 if d <= radius else 0))
    ends = {k: {"traces": n, "within_radius_of_a_node": near / float(max(n, 1))} for k, (n, near) in ends.items()}
    out = {"config": a.config, "vehicles": a.vehicles, "points": a.points, "meili": meili,
           "oracle_seconds": round(t_match, 2), "segment_id_agreement": agr["segment_id_agreement"],
           "sequences_exact": agr["sequences_exact"], "breakdown": agr["breakdown"], "columns": col,
           "trace_ends": ends}
    js = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
