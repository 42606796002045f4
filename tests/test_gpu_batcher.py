"""The native batcher on the GPU engine (BASELINE config 5's topology): its
binary fast path (SoA batches, responses written only for forwarded records),
its JSON path (the exact request bodies through otm_report_batch) and the raw
path (otm_batcher_process_raw: native formatter -> batcher -> GPU) against
the serial Python restatements -- oracle/pyformatter.py for
Formatter.format, oracle/pybatcher.py for BatchingProcessor/Batch
(BatchingProcessor.java:56-130, Batch.java:46-84) -- posting each body to the
CPU oracle's /report handler (oracle.handle_request), record at a time, as
the Java host's synchronous HttpClient.POST does (Batch.java:63).  The GPU
never checks itself here: every forwarded response is the oracle's."""
import numpy as np
import pytest

from reporter_amd import Engine
from reporter_amd.batcher import Batcher

from test_batcher import compare, make_stream, run_native, run_python

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("json_path,threads", [(False, 0), (True, 0), (False, 6), (True, 6)],
                         ids=["binary", "json", "binary_threads", "json_threads"])
def test_gpu_batcher_matches_serial_restatement(small_graph, oracle, json_path, threads):
    g = oracle.Graph(small_graph)
    recs = make_stream(small_graph, n_veh=30, n_pts=80, seed=47)
    bp = run_python(recs, lambda body: oracle.handle_request(g, body)[1])
    with Engine(graph_path=small_graph) as eng:
        nb = run_native(recs, Batcher(engine=eng, json_path=json_path, threads=threads))
        st = compare(bp, nb, recs)
        assert st["forwarded"] > 10 and st["match_batches"] < st["requests"]


@pytest.mark.parametrize("json_path", [False, True], ids=["binary", "json"])
def test_gpu_batcher_on_multi_device_engine(small_graph, oracle, json_path):
    """The batcher over a multi-device engine (two members, repeated device 0):
    each key's requests go to its murmur2 member; forwarded records, counts
    and stored batches equal the serial restatement's over the oracle."""
    g = oracle.Graph(small_graph)
    recs = make_stream(small_graph, n_veh=30, n_pts=80, seed=53)
    bp = run_python(recs, lambda body: oracle.handle_request(g, body)[1])
    with Engine(graph_path=small_graph, devices=[0, 0]) as grp:
        nb = run_native(recs, Batcher(engine=grp, json_path=json_path, threads=4))
        st = compare(bp, nb, recs)
        assert st["forwarded"] > 10


@pytest.mark.parametrize("json_path,threads", [(False, 0), (True, 0), (False, 4)],
                         ids=["binary", "json", "binary_threads"])
def test_gpu_batcher_exotic_keys(small_graph, oracle, json_path, threads):
    """Keys outside ASCII (HttpClient's ISO-8859-1 body, HttpClient.java:26): in
    binary mode a key whose body the service would reject or read differently
    takes the byte-level path; forwarded records (the 400 bodies among them),
    counts and stored batches equal the serial restatement's over the oracle."""
    from test_transport import check_exotic_keys
    g = oracle.Graph(small_graph)
    with Engine(graph_path=small_graph) as eng:
        check_exotic_keys(small_graph, lambda body: oracle.handle_request(g, body)[1],
                          Batcher(engine=eng, json_path=json_path, threads=threads))


RAW_SPECS = {
    # README.md's two layouts (the reporter-kafka --formatter argument)
    "json": ",json,id,latitude,longitude,timestamp,accuracy",
    "sv": ",sv,\\|,1,9,10,0,5,yyyy-MM-dd HH:mm:ss",
}


def raw_messages(recs, kind):
    """The records as raw messages of the given layout (plus a few the
    formatter drops), with their record timestamps in ms."""
    import datetime
    ep = datetime.datetime(1970, 1, 1)
    msgs, ts = [], []
    for i, (key, lat, lon, acc, t) in enumerate(recs):
        if kind == "json":
            msgs.append('{"timestamp":%d,"id":"%s","accuracy":%d,"latitude":%r,"longitude":%r}'
                        % (t, key, acc, lat, lon))
        else:
            msgs.append("%s|%s|x|x|x|%d|x|x|x|%r|%r|x|x|x"
                        % ((ep + datetime.timedelta(seconds=int(t))).strftime("%Y-%m-%d %H:%M:%S"), key, acc,
                           lat, lon))
        ts.append(t * 1000)
        if i % 61 == 5:
            msgs.append("not a record" if kind == "json" else "a|b")
            ts.append(t * 1000)
    return msgs, ts


def run_python_raw(msgs, ts, spec, post):
    """Formatter.format then BatchingProcessor.process per message, dropping
    what the formatter throws on (KeyedFormattingProcessor.java:30-37)."""
    from oracle import pybatcher, pyformatter
    f = pyformatter.Formatter(spec)
    bp = pybatcher.BatchingProcessor(post)
    dropped = 0
    for m, t in zip(msgs, ts):
        try:
            key, lat, lon, acc, tm = f.format(m.encode("utf-8"))
        except pyformatter.Drop:
            dropped += 1
            continue
        bp.process(key, pybatcher.Point(lat, lon, acc, tm), t)
    bp.close()
    return bp, dropped


@pytest.mark.parametrize("kind,json_path,threads", [("json", False, 4), ("json", True, 0), ("sv", False, 0),
                                                    ("sv", True, 4)],
                         ids=["json_binary", "json_jsonpath", "sv_binary", "sv_jsonpath"])
def test_gpu_batcher_process_raw_vs_oracle(small_graph, oracle, kind, json_path, threads):
    """BASELINE config 5 end to end on the GPU: raw messages through
    otm_batcher_process_raw (native formatter -> native batcher -> GPU engine)
    against pyformatter -> pybatcher -> the oracle's /report handler.  The
    forwarded (record, key, response) triples, request count, dropped count
    and store are equal; the responses are the oracle's bytes."""
    from reporter_amd.formatter import Formatter
    g = oracle.Graph(small_graph)
    recs = make_stream(small_graph, n_veh=24, n_pts=70, seed=59)
    msgs, ts = raw_messages(recs, kind)
    bp, dropped = run_python_raw(msgs, ts, RAW_SPECS[kind], lambda body: oracle.handle_request(g, body)[1])
    assert dropped > 0
    with Engine(graph_path=small_graph) as eng:
        nb = Batcher(engine=eng, json_path=json_path, threads=threads)
        fmt = Formatter(RAW_SPECS[kind])
        for i in range(0, len(msgs), 173):  # several process_raw calls, as Kafka polls deliver them
            nb.process_raw(fmt, msgs[i:i + 173], ts[i:i + 173], nthreads=3)
        nb.close()
        fwd = sorted(nb.forwarded())
        ref = sorted(bp.forwarded)
        assert len(fwd) == len(ref) and len(ref) > 10
        assert fwd == ref
        st = nb.stats()
        assert st["raw_messages"] == len(msgs) and st["raw_dropped"] == dropped
        assert st["records"] == len(msgs) - dropped
        assert st["requests"] == bp.requests
        assert st["stored_batches"] == len(bp.store)
        for key, batch in bp.store.items():
            pts, ms = nb.batch(key)
            assert np.float32(ms) == batch.max_separation
            assert [(np.float32(a), np.float32(b), c, d) for a, b, c, d in pts] == \
                [(p.lat, p.lon, p.accuracy, p.time) for p in batch.points]


def test_gpu_report_transport_bodies(small_graph, oracle):
    """The reference-recorded transport cases through otm_report and
    otm_report_batch (40 bodies: the GPU request reader takes the batch and
    hands non-ASCII uuids to the host readers): the 400 bodies are the
    reference's own, the 200 bodies the oracle's."""
    from test_transport import CASES
    g = oracle.Graph(small_graph)
    bodies = [bytes.fromhex(c["body_hex"]) for c in CASES] * 2
    want = []
    for c, b in zip(CASES * 2, bodies):
        w = oracle.handle_request(g, b)
        if c["code"] != 200:
            assert w == (c["code"], c["response"])
        want.append(w)
    with Engine(graph_path=small_graph) as eng:
        assert [eng.report(b) for b in bodies[:len(CASES)]] == want[:len(CASES)]
        assert eng.report_batch(bodies) == want
