#!/usr/bin/env python3
"""Spill statistics of tests/test_no_limits.py's batches on the GPU (which
tiers ran, how many times the batch was run): diagnostic for the no-limit
tiers.  Prints one JSON line per batch."""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import test_no_limits as T
    from reporter_amd import Engine, synth
    d = tempfile.mkdtemp()
    g = synth.make_graph(os.path.join(d, "grid32.otmg"), width_m=12000, height_m=12000, block_m=32, jitter_m=0,
                         arterial_every=8, highway_every=1000, complex_every=4, seg_max_m=300)
    b = T.grid_batch(g)
    with Engine(graph_path=g, **T.GRID_MEILI) as eng:
        print(json.dumps({"index": eng.index_info()}), flush=True)
        for r in range(2):
            eng.match(b)
            print(json.dumps({"grid_run": r, "spill": eng.spill_stats(), "stages_ms": eng.stage_ms()
                              if hasattr(eng, "stage_ms") else None}), flush=True)


if __name__ == "__main__":
    main()
