"""The GPU request reader and response writer (reporter_amd/csrc/requests.hip,
responses.hip): otm_report_batch's bodies decoded and its responses written
on the device.  A body in the Java batcher's exact form
(Batch.java:52-61, Point.java:39-45) must decode to the host reader's points
bit for bit (report.cpp fast_request, itself pinned against the DOM path in
test_fast_request.py), every other body must be left to the host readers,
and the /report responses must be byte-equal to the host readers' (OTM_GPU_JSON=0)
and to the oracle's."""
import random
import re

import numpy as np
import pytest

from reporter_amd import Engine, encode_request, synth
from test_fast_request import java_bodies, mutate, points

pytestmark = pytest.mark.gpu

NUM = r"-?(?:0|[1-9][0-9]*)(?:\.[0-9]+)?"
POINT = r'\{"lat":%s,"lon":%s,"time":%s,"accuracy":%s\}' % (NUM, NUM, NUM, NUM)
STRICT = re.compile(r'\{"uuid":"[\x20\x21\x23-\x5b\x5d-\x7e]*","trace":\[%s(?:,%s)+\]\}' % (POINT, POINT))


def _short(tok):
    """the reader's literal limits: <= 15 significant digits for a float, <= 18
    characters for an int"""
    if "." in tok:
        return len(tok.lstrip("-").replace(".", "")) <= 15
    return len(tok) <= 18


def gpu_form(body):
    """whether the GPU reader takes the body (else the host readers do)"""
    try:
        s = body.decode("ascii")
    except UnicodeDecodeError:
        return False
    if not STRICT.fullmatch(s):
        return False
    tr = s[s.index('"trace":[') + 9:-2]
    return all(_short(t) for t in re.findall(NUM, re.sub(r'"[a-z]+":', " ", tr)))


def _bodies(small_graph, n, seed, uuid="veh%d"):
    b = synth.make_traces(small_graph, n, 50, seed=seed)
    out = []
    for t in range(n):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        out.append(encode_request(uuid % t, b["lat"][a:e], b["lon"][a:e], b["time"][a:e].astype(np.int64),
                                  b["accuracy"][a:e].astype(np.int32)))
    return out


def test_gpu_reader_points_match_host_reader(small_graph):
    """Java bodies, and variants that stay in the exact form (negative zero,
    float times and accuracies, 15-digit decimals, big integers): the decoded
    batch is the host reader's points, in request order."""
    rng = random.Random(31)
    bodies = java_bodies(rng, 120)
    extra = []
    def sub(s, key, val):
        return re.sub(r'"%s":[-0-9.]+' % key, '"%s":%s' % (key, val), s, count=1)
    for b in bodies[:60]:
        s = b.decode()
        extra.append(sub(sub(s, "lat", "-0.0"), "accuracy", "-0").encode())
        extra.append(sub(sub(s, "time", "1462826734.5"), "accuracy", "5.25").encode())
        extra.append(sub(s, "lon", "-122.123456789012").encode())
        extra.append(sub(s, "time", "999999999999999999").encode())
        extra.append(sub(s, "lat", "0").encode())
    bodies += extra
    assert all(gpu_form(b) for b in bodies)
    with Engine(graph_path=small_graph) as eng:
        eng.report_batch(bodies)
        off = eng.debug("in_trace_off")
        got = [eng.debug(k) for k in ("in_lat", "in_lon", "in_time", "in_acc")]
    assert len(off) == len(bodies) + 1
    for k, body in enumerate(bodies):
        n, want = points(body, True)
        a, e = off[k], off[k + 1]
        assert e - a == n, body[:80]
        assert tuple(g[a:e].tobytes() for g in got) == want[:4], body[:80]


@pytest.mark.parametrize("writer", ["1", "0"], ids=["gpu_writer", "host_writer"])
def test_gpu_reader_mixed_bodies_byte_equal_to_host_readers(small_graph, oracle, monkeypatch, writer):
    """Java bodies mixed with mutated ones (whitespace, key orders, escapes,
    exponents, bigints, one-point traces, malformed JSON): the GPU reader takes
    exactly the exact-form bodies, and every response (code and body) equals the
    host readers' and the oracle's, in request order."""
    rng = random.Random(32)
    base = _bodies(small_graph, 90, 71)
    bodies = []
    for b in base:
        bodies.append(b)
        if rng.random() < 0.5:
            bodies.append(mutate(rng, b))
    bodies += [b"", b"[]", b"{}", b'{"uuid":"x","trace":[]}', b'{"uuid":"x","trace":[{"lat":1}]}',
               b'{"uuid":"x","trace":[{"lat":1,"lon":2,"time":3,"accuracy":4}]}',
               b'{"uuid":"x\\"y","trace":[{"lat":1,"lon":2,"time":3,"accuracy":4},{"lat":1,"lon":2,"time":9,"accuracy":4}]}',
               b'{"uuid":"x","trace":[{"lat":1,"lon":2,"time":3,"accuracy":4},{"lat":1,"lon":2,"time":9,"accuracy":4}]} ',
               b'{"uuid":"x","trace":[{"lat":1,"lon":2,"time":3,"accuracy":4},,{"lat":1,"lon":2,"time":9,"accuracy":4}]}',
               b'{"uuid":"x","trace":[{"lat":1,"lon":2,"time":3,"accuracy":4}{"lat":1,"lon":2,"time":9,"accuracy":4}]}',
               b'{"uuid":"{","trace":[{"lat":1,"lon":2,"time":3,"accuracy":4},{"lat":1.0e1,"lon":2,"time":9,"accuracy":4}]}']
    # times below the GPU writer's float range (2^-10): those bodies' floats
    # are formatted by the host writer from the typed records
    for b in base[:6]:
        cnt = iter(range(1, 10 ** 6))
        bodies.append(re.sub(r'"time":[0-9]+', lambda m: '"time":0.0000%03d' % next(cnt), b.decode()).encode())
    assert 0 < sum(map(gpu_form, bodies)) < len(bodies)
    monkeypatch.setenv("OTM_GPU_WRITE", writer)
    g = oracle.Graph(small_graph)
    with Engine(graph_path=small_graph) as eng:
        got = eng.report_batch(bodies)
        off = eng.debug("in_trace_off")
        monkeypatch.setenv("OTM_GPU_JSON", "0")
        host = eng.report_batch(bodies)
    assert got == host
    for body, cr in zip(bodies, got):
        assert cr == oracle.handle_request(g, body), body[:80]


@pytest.mark.parametrize("writer", ["1", "0"], ids=["gpu_writer", "host_writer"])
def test_gpu_reader_long_bodies_and_windows(small_graph, oracle, monkeypatch, writer):
    """traces long enough to span many of the reader's 1 KB windows, with
    points of every length, and uuids of every length up to 300 bytes"""
    b = synth.make_traces(small_graph, 40, 400, seed=73)
    bodies = []
    for t in range(40):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        bodies.append(encode_request("u" * (t * 7 + 1), b["lat"][a:e], b["lon"][a:e], b["time"][a:e].astype(np.int64),
                                     b["accuracy"][a:e].astype(np.int32)))
    assert all(gpu_form(x) for x in bodies)
    monkeypatch.setenv("OTM_GPU_WRITE", writer)
    g = oracle.Graph(small_graph)
    with Engine(graph_path=small_graph) as eng:
        got = eng.report_batch(bodies)
        assert len(eng.debug("in_trace_off")) == 41
    for body, cr in zip(bodies, got):
        assert cr == oracle.handle_request(g, body)
