"""Print the distance index each BASELINE config graph gets (radius, entries,
incomplete rows, build time).  GPU box: python scripts/index_info.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reporter_amd import Engine, synth  # noqa: E402

for c in (int(a) for a in (sys.argv[1:] or ["2", "4"])):
    g = synth.cached_graph(c)
    with Engine(graph_path=g, **synth.CONFIGS[c].get("meili", {})) as e:
        print("config", c, e.graph_info(), e.index_info(), flush=True)
