#!/usr/bin/env python3
"""How often does a turn-aware route choice change the match?

SURVEY Appendix B picks a transition's route by "distance cost plus turn
penalty"; the spec (oracle and GPU) picks the distance-shortest route and adds
its turn cost.  The oracle's experiment switch (orc_params.turn_aware) runs an
edge-labelled search instead -- a label per (node, incoming edge), minimising
distance + turn units / 64.  This script matches the same synthetic traces both
ways and counts what changes: transition costs, Viterbi states, and per trace
the OSMLR segment-id sequence and the full segment records.  CPU only.

  python scripts/turn_aware_rate.py [--vehicles-c2 2000] [--vehicles-c4 1000] [--out profiles/r03_turn_aware_rate.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import pyoracle  # noqa: E402
from reporter_amd import synth  # noqa: E402


def compare(graph, batch, meili, nthreads):
    g = pyoracle.Graph(graph)
    t0 = time.time()
    a = pyoracle.match_batch(g, batch, p=pyoracle.params(**meili), keep_stages=True, nthreads=nthreads)
    t1 = time.time()
    b = pyoracle.match_batch(g, batch, p=pyoracle.params(turn_aware=1, **meili), keep_stages=True,
                             nthreads=nthreads)
    t2 = time.time()
    ta, tb = a["trans"], b["trans"]
    fin_a, fin_b = np.isfinite(ta), np.isfinite(tb)
    diff_t = int(((ta != tb) & (fin_a | fin_b)).sum())
    n_t = int((fin_a | fin_b).sum())
    col = a["ncand"] > 0
    diff_state = int((a["state"] != b["state"])[col].sum())
    tr_a, tr_b = a["traces"], b["traces"]
    seq = rec = 0
    nt = len(tr_a)
    for t in range(nt):
        sa = a["segments"][tr_a["seg_off"][t]:tr_a["seg_off"][t] + tr_a["seg_cnt"][t]]
        sb = b["segments"][tr_b["seg_off"][t]:tr_b["seg_off"][t] + tr_b["seg_cnt"][t]]
        ida, idb = sa["segment_id"], sb["segment_id"]
        seq += int(not np.array_equal(ida[ida >= 0], idb[idb >= 0]))
        keys = ("segment_id", "start_time", "end_time", "length", "begin_shape_index", "end_shape_index")
        rec += int(len(sa) != len(sb) or any(not np.array_equal(sa[k], sb[k]) for k in keys))
    return {"points": int(len(batch["lat"])), "traces": nt,
            "transitions_compared": n_t, "transitions_changed": diff_t,
            "transitions_changed_frac": diff_t / max(n_t, 1),
            "column_states_changed": diff_state, "columns": int(col.sum()),
            "column_states_changed_frac": diff_state / max(int(col.sum()), 1),
            "traces_segment_id_sequence_changed": seq, "traces_segment_id_sequence_changed_frac": seq / max(nt, 1),
            "traces_segment_records_changed": rec, "traces_segment_records_changed_frac": rec / max(nt, 1),
            "oracle_seconds": {"spec": t1 - t0, "turn_aware": t2 - t1}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vehicles-c2", type=int, default=2000)
    ap.add_argument("--vehicles-c4", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_turn_aware_rate.json"))
    args = ap.parse_args()
    out = {"what": "spec (distance-shortest route + its turn cost) vs turn-aware route choice (distance + turn "
                   "cost minimised, label per (node, incoming edge)), CPU oracle, same traces",
           "turn_penalty_factor": 200.0}
    for cfg, nv in ((2, args.vehicles_c2), (4, args.vehicles_c4)):
        c = synth.CONFIGS[cfg]
        graph = synth.cached_graph(cfg)
        tr = dict(c["traces"])
        tr["n_vehicles"] = nv
        b = synth.make_traces(graph, **tr)
        r = compare(graph, b, dict(c.get("meili", {})), args.threads)
        out["config%d" % cfg] = r
        print("config %d: %s" % (cfg, json.dumps(r)), flush=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
