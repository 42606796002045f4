"""Multi-device engine (otm_engine_create with ndev > 1, reporter_amd/csrc/group.cpp).

One host process driving several GPUs through one handle, as the Java host
(one JVM, Batch.java:63) would: traces go to member (murmur2(uuid) &
0x7fffffff) % ndev, Kafka's partition of the key, the
members run concurrently and the results come back merged in request order.
The box has one GPU, so the members are repeated device 0 (each a full graph
and index replica on it): the split, the concurrent members and the merge are
what is checked, byte-equal to one engine and to the CPU oracle.
"""
import threading

import numpy as np
import pytest

from reporter_amd import Engine, _lib, encode_request, synth
from reporter_amd.engine import OtmError

pytestmark = pytest.mark.gpu

KEYS = ("traces", "segments", "reports", "way_ids")


def _bodies(b, n, prefix="veh"):
    out = []
    for t in range(n):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        out.append(encode_request("%s%d" % (prefix, t), b["lat"][a:e], b["lon"][a:e],
                                  b["time"][a:e].astype(np.int64), b["accuracy"][a:e].astype(np.int32)))
    return out


@pytest.mark.parametrize("ndev", [2, 3])
def test_group_report_batch_byte_equal(small_graph, oracle, ndev):
    b = synth.make_traces(small_graph, 90, 60, seed=71)
    bodies = _bodies(b, 90)
    bodies += [b"", b"[]", b'{"uuid":"x","trace":[]}', b'{"uuid":7,"trace":[{"lat":1}]}']
    g = oracle.Graph(small_graph)
    with Engine(graph_path=small_graph, devices=[0] * ndev) as grp, Engine(graph_path=small_graph) as one:
        assert grp.members() == ndev and one.members() == 1
        got = grp.report_batch(bodies)
        assert got == one.report_batch(bodies)
        for body, (code, resp) in zip(bodies, got):
            assert (code, resp) == oracle.handle_request(g, body), body[:80]
        # every member got work: the uuids spread over all of them
        shards = {_lib.lib().otm_murmur2(("veh%d" % t).encode(), len("veh%d" % t)) & 0x7FFFFFFF for t in range(90)}
        assert len({s % ndev for s in shards}) == ndev
        assert grp.report(bodies[3]) == got[3]
        assert grp.match_json(bodies[5]) == one.match_json(bodies[5])


def test_group_match_soa_merge(small_graph, oracle, results_equal):
    """The binary batch is split into point-balanced contiguous ranges and
    merged back: every array equal to one engine's and to the oracle's."""
    b = synth.make_traces(small_graph, 257, 70, seed=73)
    orc = oracle.match_batch(oracle.Graph(small_graph), b, nthreads=8)
    with Engine(graph_path=small_graph, devices=[0, 0, 0]) as grp, Engine(graph_path=small_graph) as one:
        r = grp.match(b)
        r1 = one.match(b)
        for k in KEYS:
            assert getattr(r, k).tobytes() == getattr(r1, k).tobytes(), k
        results_equal(orc, r, "group")
        again = grp.fetch()
        for k in KEYS:
            assert getattr(again, k).tobytes() == getattr(r, k).tobytes(), k
        # empty batch
        e = grp.match({"trace_off": np.zeros(1, np.int64), "lat": np.zeros(0, np.float32),
                       "lon": np.zeros(0, np.float32), "time": np.zeros(0), "accuracy": np.zeros(0, np.float32)})
        assert len(e.traces) == 0


def test_group_submit_poll_and_threads(small_graph):
    """Async submit/poll and 4 host threads on one multi-device engine, with
    repeated uuids: results byte-equal to the sequential ones."""
    b = synth.make_traces(small_graph, 48, 50, seed=79)
    bodies = _bodies(b, 48, prefix="car") + _bodies(b, 48, prefix="car")
    with Engine(graph_path=small_graph, devices=[0, 0]) as grp:
        want = grp.report_batch(bodies)
        for k, body in enumerate(bodies):
            grp.submit(body, k)
        seen = {}
        while len(seen) < len(bodies):
            for tag, code, resp in grp.poll(256, 2000000):
                seen[tag] = (code, resp)
        assert [seen[k] for k in range(len(bodies))] == want
        got = {}

        def run(i):
            got[i] = [grp.report(x) for x in bodies[i::4]]
        th = [threading.Thread(target=run, args=(i,)) for i in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for i in range(4):
            assert got[i] == want[i::4]


def test_group_members_and_device_calls(small_graph):
    import torch
    b = synth.make_traces(small_graph, 64, 40, seed=83)
    with Engine(graph_path=small_graph, devices=[0, 0]) as grp:
        assert grp.graph_info() == grp.member(1).graph_info()
        # device-side calls belong to a member
        with pytest.raises(OtmError):
            grp.hist_bind(torch.zeros(16, dtype=torch.int32, device="cuda:0"), 16, 10.0)
        with pytest.raises(OtmError):
            grp.clone()
        m = grp.member(1)
        r = m.match(b)
        r0 = grp.match(b)
        assert len(r.traces) == len(r0.traces) == 64
        assert r.segments.tobytes() == r0.segments.tobytes()
        with pytest.raises(OtmError):
            grp.member(2)
