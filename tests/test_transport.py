"""The /report transport's charset steps (missing item of VERDICT r3 #3).

The reference sends a Java String body through new StringEntity(body)
(HttpClient.java:26), whose default charset is ISO-8859-1: a character above
U+00FF becomes '?', U+0080..U+00FF a single byte.  reporter_service.py then
runs body.decode('utf-8') (py/reporter_service.py:99), so a uuid holding a
Latin-1 character gets a 400.  The uuid is the Kafka record key
(Batch.java:55, unescaped), which the batcher received through
StringDeserializer (JDK 8 UTF-8 decoding with U+FFFD replacement).

Pinned by tests/golden/transport_cases.json: the reference service's own
answers to the bytes HttpClient would send for each key (make_golden.py).
The Java charset steps themselves (no JVM here) are restated in
reporter_amd/csrc/javastr.cpp and, independently, in oracle/pyformatter.py /
tests/golden/make_golden.py; the hand-worked JDK 8 decoder cases below follow
sun.nio.cs.UTF_8's rules.
"""
import json
import os

import numpy as np
import pytest

from reporter_amd import engine as E
from reporter_amd.batcher import Batcher

GOLD = os.path.join(os.path.dirname(__file__), "golden")
with open(os.path.join(GOLD, "transport_cases.json")) as f:
    CASES = json.load(f)

# the two points of make_golden.TRANSPORT_TRACE (exact in float32)
LAT = [14.5, 14.5]
LON = [121.25, 121.5]
TIME = [1000, 1010]
ACC = [5, 5]


def wire_of(key_bytes):
    """The key's bytes inside the body the product encoder writes."""
    body = E.encode_request(key_bytes, [], [], [], [])
    assert body.startswith(b'{"uuid":"') and body.endswith(b'","trace":]}')
    return body[9:-12]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_request_bytes_are_httpclients(case):
    """otm_encode_request(kafka key bytes) == the bytes HttpClient sends."""
    key = bytes.fromhex(case["key_utf8_hex"])
    assert E.encode_request(key, LAT, LON, TIME, ACC) == bytes.fromhex(case["body_hex"])


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_reference_answer_to_transport_bytes(case, oracle):
    """The oracle and the product's host path answer those bytes as the
    reference did (the 400s of body.decode('utf-8') / json.loads, the 200s)."""
    body = bytes.fromhex(case["body_hex"])
    code, resp, _ = oracle.report_segments(body, '{"segments":[]}')
    assert (code, resp) == (case["code"], case["response"])
    code, resp = E.report_segments(body, '{"segments":[]}')
    assert (code, resp) == (case["code"], case["response"])


# Hand-worked JDK 8 cases: key bytes -> String (StringDeserializer) -> ISO-8859-1
JDK_DECODE = [
    (b"\xc3\xa9", b"\xe9"),
    (b"\xed\xa0\x80", b"?"),          # an encoded surrogate: ONE U+FFFD (Python's 'replace' gives three)
    (b"\xed\xa0", b"?"),              # truncated surrogate lead: one
    (b"\xed\xa0A", b"?A"),            # malformedN(3) = 2
    (b"\xe0\x80\x80", b"???"),        # overlong: 1 + 1 + 1
    (b"\xc3", b"?"),
    (b"\xc3A", b"?A"),
    (b"\xf0\x9f\x98\x80", b"?"),      # U+1F600: a surrogate pair, one '?'
    (b"\xf0\x9f\x98", b"?"),          # truncated 4-byte form at the end
    (b"\xf0\x9fA", b"?A"),
    (b"\xf4\x90\x80\x80", b"????"),   # above U+10FFFF
    (b"\xf5\x80", b"??"),
    (b"\xff", b"?"),
    (b"\xc0\xaf", b"??"),
    (b"a\xe9b", b"a?b"),
    (b"\xe6\x97\xa5", b"?"),
    (b"\xc2\xa0", b"\xa0"),
    (b"plain-ascii_01", b"plain-ascii_01"),
]


@pytest.mark.parametrize("raw,wire", JDK_DECODE, ids=lambda v: v.hex() if isinstance(v, bytes) else str(v))
def test_kafka_key_to_wire_jdk8(raw, wire):
    assert wire_of(raw) == wire


def test_python_restatement_of_jdk_decoder_agrees():
    """oracle/pyformatter.java_utf8_decode (the independent restatement) gives
    the same Strings on the hand cases and on random byte strings."""
    from oracle import pyformatter as P
    for raw, wire in JDK_DECODE:
        assert P.java_latin1(P.java_utf8_decode(raw)) == wire
    rng = np.random.default_rng(3)
    alphabet = np.array([0x41, 0x7F, 0x80, 0x9F, 0xA0, 0xBF, 0xC2, 0xC3, 0xDF, 0xE0, 0xE1, 0xED, 0xEF, 0xF0, 0xF4,
                         0xF5, 0xFF, 0x90, 0x8F], np.uint8)
    for _ in range(3000):
        raw = bytes(rng.choice(alphabet, size=int(rng.integers(1, 9))).tolist())
        assert wire_of(raw) == P.java_latin1(P.java_utf8_decode(raw)), raw.hex()


def exotic_keys():
    """Record keys as the formatted topic carries them (StringSerializer's UTF-8)."""
    ks = [c for c in CASES if c["name"] != "ascii"]
    out = [bytes.fromhex(c["key_utf8_hex"]) for c in ks]
    out += [b"\xff\xfe", b"\xfe", "Ａ".encode(), "\U0001F600z".encode()]  # the first two are one Java key
    return out


def check_exotic_keys(graph, post, batcher):
    """Run a stream whose vehicles carry exotic_keys() through the serial
    restatement (post(body) -> response) and the native batcher; the same
    forwarded (record, key, response) triples -- the 400 bodies forwarded and
    their batches cleared -- the same request count and the same store."""
    from oracle import pybatcher
    from oracle.pyformatter import java_utf8_decode
    from tests.test_batcher import make_stream, run_native
    keys = exotic_keys()
    recs = make_stream(graph, n_veh=len(keys) + 2, n_pts=40, seed=61)
    ids = sorted({r[0] for r in recs})
    kmap = {v: (keys[i] if i < len(keys) else v.encode()) for i, v in enumerate(ids)}
    nrecs = [(kmap[r[0]],) + r[1:] for r in recs]
    bp = pybatcher.BatchingProcessor(post)
    for key, lat, lon, acc, t in nrecs:
        bp.process(java_utf8_decode(key), pybatcher.Point(lat, lon, acc, t), t * 1000)
    bp.close()
    nb = run_native(nrecs, batcher)
    fwd = sorted(nb.forwarded())
    ref = sorted(bp.forwarded)
    assert fwd == ref
    assert any(r.startswith('{"error":"\'utf-8\' codec') for _, _, r in ref)
    assert any(r.startswith('{"stats"') for _, _, r in ref)
    st = nb.stats()
    assert st["requests"] == bp.requests
    assert st["stored_batches"] == len(bp.store)
    for key, batch in bp.store.items():
        got = nb.batch(key.encode("utf-8"))
        assert got is not None
        assert [(np.float32(a), np.float32(b), c, d) for a, b, c, d in got[0]] == \
            [(p.lat, p.lon, p.accuracy, p.time) for p in batch.points]


@pytest.mark.parametrize("threads", [0, 3])
def test_batcher_with_exotic_keys_matches_serial_restatement(small_graph, oracle, threads):
    """Handler = the oracle's byte-level /report."""
    g = oracle.Graph(small_graph)
    check_exotic_keys(small_graph, lambda body: oracle.handle_request(g, body)[1],
                      Batcher(handler=lambda bodies: [oracle.handle_request(g, x) for x in bodies], threads=threads))


def test_serial_restatement_treemap_order_is_utf16():
    """The serial restatement's close() walks the store in String.compareTo
    order (BatchingProcessor.java:120-130): U+1F600 (surrogates D83D DE00)
    sorts before U+FF21 in Java, after it by code point or UTF-8 bytes.  (The
    native batcher answers every key's close() report in one matcher round,
    whose results do not depend on the order.)"""
    import re
    from oracle import pybatcher

    def first_lat(body):
        return float(re.search(rb'"lat":([0-9.]+)', body).group(1))

    keys = ["\uff21", "\U0001F600", "b", "\u00e9"]
    lats = [37.0, 37.25, 37.5, 37.75]  # one per key, exact in float32
    got = []
    bp = pybatcher.BatchingProcessor(lambda body: got.append(first_lat(body)) or '{"segments":[]}')
    for ts in (1000, 1001):
        for k, la in zip(keys, lats):
            bp.process(k, pybatcher.Point(la, -122.0, 5, ts), ts * 1000)
    bp.close()
    assert got == [37.5, 37.75, 37.25, 37.0]  # b < U+00E9 < U+1F600 < U+FF21
