"""The native batcher on the GPU engine: its binary fast path (SoA batches,
responses written only for forwarded records) and its JSON path (the exact
request bodies through otm_report_batch) against the serial Python
restatement of BatchingProcessor posting each body to Engine.report."""
import pytest

from reporter_amd import Engine
from reporter_amd.batcher import Batcher

from test_batcher import compare, make_stream, run_native, run_python

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("json_path,threads", [(False, 0), (True, 0), (False, 6), (True, 6)],
                         ids=["binary", "json", "binary_threads", "json_threads"])
def test_gpu_batcher_matches_serial_restatement(small_graph, json_path, threads):
    recs = make_stream(small_graph, n_veh=30, n_pts=80, seed=47)
    with Engine(graph_path=small_graph) as eng:
        bp = run_python(recs, lambda body: eng.report(body)[1])
        nb = run_native(recs, Batcher(engine=eng, json_path=json_path, threads=threads))
        st = compare(bp, nb, recs)
        assert st["forwarded"] > 10 and st["match_batches"] < st["requests"]


@pytest.mark.parametrize("json_path", [False, True], ids=["binary", "json"])
def test_gpu_batcher_on_multi_device_engine(small_graph, json_path):
    """The batcher over a multi-device engine (two members, repeated device 0):
    each key's requests go to its murmur2 member; forwarded records, counts
    and stored batches equal the serial restatement's."""
    recs = make_stream(small_graph, n_veh=30, n_pts=80, seed=53)
    with Engine(graph_path=small_graph) as one, Engine(graph_path=small_graph, devices=[0, 0]) as grp:
        bp = run_python(recs, lambda body: one.report(body)[1])
        nb = run_native(recs, Batcher(engine=grp, json_path=json_path, threads=4))
        st = compare(bp, nb, recs)
        assert st["forwarded"] > 10


@pytest.mark.parametrize("json_path,threads", [(False, 0), (True, 0), (False, 4)],
                         ids=["binary", "json", "binary_threads"])
def test_gpu_batcher_exotic_keys(small_graph, json_path, threads):
    """Keys outside ASCII (HttpClient's ISO-8859-1 body, HttpClient.java:26): in
    binary mode a key whose body the service would reject or read differently
    takes the byte-level path; forwarded records (the 400 bodies among them),
    counts and stored batches equal the serial restatement's."""
    from test_transport import check_exotic_keys
    with Engine(graph_path=small_graph) as eng:
        check_exotic_keys(small_graph, lambda body: eng.report(body)[1],
                          Batcher(engine=eng, json_path=json_path, threads=threads))


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
