"""The native batcher (otm_batcher, BatchingProcessor + Batch restated in C++)
against the serial Python restatement in oracle/pybatcher.py.

The native batcher runs every key's operations in the reference's serial
order but sends the requests of all ready keys to the matcher together; the
Python one runs record by record with a synchronous matcher, as the Java host
does.  Same stream, same matcher => the same forwarded (record, key, response)
triples, the same requests, the same final store.  CPU: the matcher is the
CPU oracle's /report handler; GPU (test_gpu_batcher.py): the engine.
"""
import numpy as np
import pytest

from reporter_amd import synth
from reporter_amd.batcher import Batcher


def make_stream(graph, n_veh=24, n_pts=70, seed=41):
    """Interleaved records (key, lat, lon, accuracy, time, ts_ms) ordered by
    record time, with session gaps and an off-network vehicle."""
    b = synth.make_traces(graph, n_veh, n_pts, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=seed)
    recs = []
    for v in range(n_veh):
        a, e = b["trace_off"][v], b["trace_off"][v + 1]
        for k, i in enumerate(range(a, e)):
            t = int(b["time"][i]) + 3 * v
            if v % 5 == 1 and k >= n_pts // 2:
                t += 150  # idle longer than the session gap, then resume
            lat, lon = float(b["lat"][i]), float(b["lon"][i])
            if v == 3:
                lat += 0.5  # off the network: empty matches, shape_used None -> batch cleared
            recs.append(("veh%02d" % v, lat, lon, int(np.ceil(b["accuracy"][i])), t))
    recs.sort(key=lambda r: (r[4], r[0]))
    return recs


def run_python(recs, post):
    from oracle import pybatcher
    bp = pybatcher.BatchingProcessor(post)
    for key, lat, lon, acc, t in recs:
        bp.process(key, pybatcher.Point(lat, lon, acc, t), t * 1000)
    bp.close()
    return bp


def run_native(recs, batcher, chunk=97):
    for i in range(0, len(recs), chunk):
        part = recs[i:i + chunk]
        batcher.process([r[0] for r in part], [r[1] for r in part], [r[2] for r in part], [r[3] for r in part],
                        [r[4] for r in part], [r[4] * 1000 for r in part])
    batcher.close()
    return batcher


def compare(bp, nb, recs):
    fwd = sorted(nb.forwarded())
    ref = sorted((s, k, r) for s, k, r in bp.forwarded)
    assert len(fwd) == len(ref)
    for a, b in zip(fwd, ref):
        assert a == b
    st = nb.stats()
    assert st["records"] == len(recs)
    assert st["requests"] == bp.requests
    assert st["null_batch_in_clean"] == bp.null_batch_in_clean
    assert st["stored_batches"] == len(bp.store)
    for key, batch in bp.store.items():
        got = nb.batch(key)
        assert got is not None
        pts, ms = got
        assert np.float32(ms) == batch.max_separation
        assert [(np.float32(a), np.float32(b), c, d) for a, b, c, d in pts] == \
            [(p.lat, p.lon, p.accuracy, p.time) for p in batch.points]
    return st


@pytest.mark.parametrize("threads", [0, 4])
def test_native_batcher_matches_serial_restatement(small_graph, oracle, threads):
    g = oracle.Graph(small_graph)
    post = lambda body: oracle.handle_request(g, body)[1]  # noqa: E731
    recs = make_stream(small_graph)
    bp = run_python(recs, post)
    nb = run_native(recs, Batcher(handler=lambda bodies: [oracle.handle_request(g, x) for x in bodies],
                                  threads=threads))
    st = compare(bp, nb, recs)
    # the stream exercised every path: gated reports, relaxed clean() reports,
    # emptied batches, the reference's clean() null case, close()
    assert st["forwarded"] > 10 and st["clean_ops"] > 100 and st["close_ops"] > 0, st
    assert bp.null_batch_in_clean > 0
    assert st["match_batches"] < st["requests"]  # requests of several keys shared matcher calls


@pytest.mark.parametrize("max_batch,threads", [(1, 0), (5, 0), (5, 3)])
def test_native_batcher_batch_limits(small_graph, oracle, max_batch, threads):
    g = oracle.Graph(small_graph)
    recs = make_stream(small_graph, n_veh=10, n_pts=40, seed=43)
    bp = run_python(recs, lambda body: oracle.handle_request(g, body)[1])
    nb = run_native(recs, Batcher(handler=lambda bodies: [oracle.handle_request(g, x) for x in bodies],
                                  max_batch=max_batch, threads=threads), chunk=13)
    compare(bp, nb, recs)


def test_request_bytes_match_java_encoding():
    """Point.Serder.put_json + Batch.report's body (Batch.java:52-61) from the
    restatement agree with the product encoder on awkward values."""
    from oracle import pybatcher
    from reporter_amd import encode_request
    vals = [37.98, -0.5, 0.0, 1.0000005, 14.543087, 121.021019, -122.4194155, 0.0000004, -0.0000006, 179.9999995]
    b = pybatcher.Batch()
    for i, v in enumerate(vals):
        b.points.append(pybatcher.Point(v, -v / 2, i, 1500000000 + i))
    got = encode_request("k1", [p.lat for p in b.points], [p.lon for p in b.points], [p.time for p in b.points],
                         [p.accuracy for p in b.points])
    assert got == b.body("k1")


def test_gates_and_trim_unit():
    """Batch.report gates (Batch.java:48-50) and the shape_used trim (:64-76)."""
    from oracle import pybatcher
    resp = {"v": '{"stats":{},"shape_used":3,"segment_matcher":{}}'}
    b = pybatcher.Batch(pybatcher.Point(37.0, -122.0, 5, 1000))
    for i in range(1, 12):
        b.update(pybatcher.Point(37.0 + 0.001 * i, -122.0, 5, 1000 + 10 * i))
    assert b.max_separation > 1000
    assert b.report("k", lambda body: resp["v"], 500, 10, 60) is not None
    assert len(b.points) == 9
    resp["v"] = '{"error":"boom"}'  # no shape_used: everything trimmed
    assert b.report("k", lambda body: resp["v"], 0, 2, 0) is not None and b.points == []


def test_quantize_decimal6_matches_text_round_trip():
    """otm_quantize_decimal6 (string-free) == float(DecimalFormat text) on
    coordinates, exact ties (k/128: HALF_EVEN at the 7th digit), signed zeros
    and values past the shortcut's range."""
    import ctypes as C
    from oracle import pybatcher
    from reporter_amd._lib import lib
    rng = np.random.default_rng(5)
    v = np.concatenate([rng.uniform(-180, 180, 20000), rng.uniform(-1e-5, 1e-5, 2000),
                        np.arange(-4096, 4096) / 128.0, np.arange(-300, 300) / 1024.0,
                        [0.0, -0.0, 5e-7, -5e-7, 1.5e-6, 2.5e-6, 1e9, -3e10, 1e30, 179.9999995]]).astype(np.float32)
    out = np.empty_like(v)
    lib().otm_quantize_decimal6(v.ctypes.data, out.ctypes.data, C.c_int64(len(v)))
    want = np.array([np.float32(float(pybatcher.decimal6(x) or "0")) for x in v.tolist()], np.float32)
    assert np.array_equal(out.view(np.uint32), want.view(np.uint32))


def test_request_bytes_match_java_encoding_wide():
    """The integer-digit DecimalFormat text against Decimal HALF_EVEN over
    coordinates, 7th-digit ties, tiny and signed-zero values, and values past
    the integer shortcut."""
    from oracle import pybatcher
    from reporter_amd import encode_request
    rng = np.random.default_rng(9)
    v = np.concatenate([rng.uniform(-180, 180, 3000), rng.uniform(-2e-6, 2e-6, 500), np.arange(-512, 512) / 128.0,
                        [0.0, -0.0, 5e-7, -5e-7, 1.5e-6, 2.5e-6, 1e9, -3e10, 1e30, 999999.5]]).astype(np.float32)
    b = pybatcher.Batch()
    for i in range(0, len(v) - 1, 2):
        b.points.append(pybatcher.Point(v[i], v[i + 1], i % 7, 1500000000 + i))
    got = encode_request("k2", [p.lat for p in b.points], [p.lon for p in b.points], [p.time for p in b.points],
                         [p.accuracy for p in b.points])
    assert got == b.body("k2")


def test_threaded_batcher_large_calls(small_graph, oracle):
    """Calls above the parallel key-lookup threshold (16k records), with a
    4-thread batcher, against the serial restatement."""
    g = oracle.Graph(small_graph)
    recs = make_stream(small_graph, n_veh=300, n_pts=70, seed=49)
    assert len(recs) > 16384
    bp = run_python(recs, lambda body: oracle.handle_request(g, body)[1])
    nb = run_native(recs, Batcher(handler=lambda bodies: [oracle.handle_request(g, x) for x in bodies], threads=4,
                                  max_pending=50000), chunk=20000)
    compare(bp, nb, recs)


@pytest.mark.parametrize("threads", [0, 3])
def test_handler_failure_is_a_null_response(small_graph, oracle, threads):
    """A /report handler that fails as a whole (HttpClient.POST's transport
    failure, HttpClient.java:37-39) answers every request of that call with
    null: Batch.report clears the batch (Batch.java:77-81) and process()
    forwards nothing (BatchingProcessor.java:70-71).  The drain goes on with
    the next calls.  The serial restatement gets None for exactly the requests
    the failing call carried."""
    g = oracle.Graph(small_graph)
    recs = make_stream(small_graph, n_veh=16, n_pts=60, seed=47)
    calls = {"n": 0}
    failed = set()

    def handler(bodies):
        calls["n"] += 1
        if calls["n"] in (2, 5):
            failed.update(bodies)
            return None
        return [oracle.handle_request(g, x) for x in bodies]

    nb = run_native(recs, Batcher(handler=handler, max_batch=7, threads=threads), chunk=31)
    assert failed, "the stream never reached a second matcher call"
    bp = run_python(recs, lambda body: None if body in failed else oracle.handle_request(g, body)[1])
    st = compare(bp, nb, recs)
    assert st["null_responses"] == len(failed)


@pytest.mark.parametrize("threads", [0, 4])
def test_native_oracle_handler_equals_python_handler(small_graph, oracle, threads):
    """The C oracle's /report handler as a C callback (orc_batcher_handler,
    the config-5 CPU baseline's matcher) against the serial restatement."""
    g = oracle.Graph(small_graph)
    recs = make_stream(small_graph, n_veh=20, n_pts=60, seed=67)
    bp = run_python(recs, lambda body: oracle.handle_request(g, body)[1])
    hh = oracle.BatcherHandler(g, nthreads=3)
    nb = run_native(recs, Batcher(native_handler=(hh.fn, hh.ctx_ptr), threads=threads))
    st = compare(bp, nb, recs)
    assert st["forwarded"] > 5
