"""GPU parity at BASELINE's full per-GPU sizes (configs 2, 3 and 4), each
batch compared field by field with the CPU oracle over every trace, plus
size-independent properties: determinism across runs and across batch
splits, and the uuid shard partition of config 3.

  config 2  the bench batch: 10k vehicles x 100 points (1M points)
  config 3  one GPU's shard of the metro run: 1M vehicles / 8 GPUs x 100
            points (12.5M points) on the 100 x 100 km graph
  config 4  state-scale graph (500 x 500 km, highway-heavy), 30 s sampling,
            sigma 50 m, radius 200 m: 20k vehicles x 100 points
"""
import os

import numpy as np
import pytest

from reporter_amd import Engine, murmur2_partition, synth

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)


def _bytes(r):
    return [getattr(r, k).tobytes() for k in ("traces", "segments", "reports", "way_ids")]


def _check_vs_oracle(oracle, results_equal, graph, batch, res, meili=None):
    orc = oracle.match_batch(oracle.Graph(graph), batch, p=oracle.params(**(meili or {})), nthreads=NTHREADS)
    results_equal(orc, res, "full batch")


def test_config2_full_batch(oracle, results_equal):
    graph = synth.cached_graph(2)
    b = synth.make_traces(graph, **synth.CONFIGS[2]["traces"])
    with Engine(graph_path=graph) as eng:
        res = eng.match(b)
        _check_vs_oracle(oracle, results_equal, graph, b, res)
        assert (res.traces["code"] == 200).mean() > 0.99
        # the same traces split over three batches give the same bytes
        parts = [synth.slice_batch(b, a, e) for a, e in ((0, 3000), (3000, 7000), (7000, 10000))]
        got = [eng.match(pb) for pb in parts]
        for pb, r in zip(parts, got):
            _check_vs_oracle(oracle, results_equal, graph, pb, r)


def test_config3_gpu_shard(oracle, results_equal):
    """One GPU's uuid shard of config 3 (Kafka murmur2 partitioner over 8
    GPUs), 12.5M points in one batch."""
    graph = synth.cached_graph(3)
    tr = dict(synth.CONFIGS[3]["traces"])
    world = 8
    ids = synth.shard_vehicle_ids(tr["n_vehicles"] // world, 0, world)
    # the shard is the murmur2 partition of the vehicle keys ("veh<id>")
    assert all(murmur2_partition("veh%d" % int(v), world) == 0 for v in ids[:1000])
    tr["n_vehicles"] = len(ids)
    b = synth.make_traces(graph, vehicle_ids=ids, **tr)
    assert 11_000_000 < len(b["lat"]) < 14_000_000
    with Engine(graph_path=graph) as eng:
        r1 = eng.match(b)
        _check_vs_oracle(oracle, results_equal, graph, b, r1)
        assert (r1.traces["code"] == 200).mean() > 0.99
        first = _bytes(r1)
        del r1
        assert _bytes(eng.match(b)) == first  # deterministic at full size


def test_config4_state_graph(oracle, results_equal):
    graph = synth.cached_graph(4)
    tr = dict(synth.CONFIGS[4]["traces"], n_vehicles=20000)
    meili = synth.CONFIGS[4]["meili"]
    b = synth.make_traces(graph, **tr)
    with Engine(graph_path=graph, **meili) as eng:
        res = eng.match(b)
        _check_vs_oracle(oracle, results_equal, graph, b, res, meili)
        assert (res.traces["code"] == 200).mean() > 0.95
        # the index radius sized from the graph covers config 4's long
        # transitions (30 s sampling): no column falls to the online tiers
        assert eng.index_info()["radius_m"] >= 5000.0
        sp = eng.spill_stats()
        assert sp["trans_online"] == 0 and sp["route_online"] == 0, sp


@pytest.mark.parametrize("budget", ["dense", "shrunk"])
def test_config3_shard_index_budget(oracle, results_equal, monkeypatch, budget):
    """Config 3's shard under an HBM budget the fast route index (30 % load,
    53 B per entry) does not fit: "dense" leaves room for the 40 % tables (40 B
    per entry) at the full radius, "shrunk" for neither, so the radius is cut
    and the columns past it go to the online search tiers.  Bit-identical to
    the oracle either way."""
    graph = synth.cached_graph(3)
    tr = dict(synth.CONFIGS[3]["traces"])
    ids = synth.shard_vehicle_ids(tr["n_vehicles"] // 8, 0, 8)[:40000]  # 4M points of the shard
    tr["n_vehicles"] = len(ids)
    b = synth.make_traces(graph, vehicle_ids=ids, **tr)
    with Engine(graph_path=graph) as eng:
        full = dict(eng.index_info(), **eng.index_tables())
    assert full["load_pct"] == 30
    # the full index's tables take ~53 B per entry at 30 % load, ~40 B at 40 %
    per_entry = 46 if budget == "dense" else 20
    monkeypatch.setenv("OTM_INDEX_BUDGET_MB", str(full["entries"] * per_entry >> 20))
    with Engine(graph_path=graph) as eng:
        info = dict(eng.index_info(), **eng.index_tables())
        assert info["load_pct"] == 40
        if budget == "dense":
            assert info["radius_m"] == full["radius_m"] and info["entries"] == full["entries"]
            assert info["bytes"] < full["bytes"]
        else:
            assert 100.0 <= info["radius_m"] < full["radius_m"]
        res = eng.match(b)
        sp = eng.spill_stats()
        if budget == "shrunk":
            assert sp["trans_online"] > 0 and sp["route_online"] > 0, sp
        _check_vs_oracle(oracle, results_equal, graph, b, res)
