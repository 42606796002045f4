"""The DOM-free reader of the Java batcher's request bytes (otm::fast_request,
reporter_amd/csrc/report.cpp) against the DOM path (parse_request +
extract_points, py/reporter_service.py:85-106,218-234): every body the fast
reader accepts must give the DOM path's points bit for bit and its uuid, and
every body outside its grammar must be handed back (-2), never misread."""
import ctypes as C
import random

import numpy as np
import pytest

from reporter_amd import _lib, encode_request

MAXP = 512


def points(body, fast):
    L = _lib.lib()
    lat = np.zeros(MAXP, np.float32)
    lon = np.zeros(MAXP, np.float32)
    tm = np.zeros(MAXP, np.float64)
    acc = np.zeros(MAXP, np.float32)
    uuid = C.create_string_buffer(256)
    n = L.otm_request_points(body, len(body), 1 if fast else 0, lat.ctypes.data, lon.ctypes.data, tm.ctypes.data,
                             acc.ctypes.data, MAXP, uuid, 256)
    if n < 0:
        return n, None
    return n, (lat[:n].tobytes(), lon[:n].tobytes(), tm[:n].tobytes(), acc[:n].tobytes(), uuid.value)


def java_bodies(rng, count):
    out = []
    for k in range(count):
        n = rng.randint(2, 60)
        lat = np.float32(37.0) + np.asarray([rng.uniform(-0.5, 0.5) for _ in range(n)], np.float32)
        lon = np.float32(-122.0) + np.asarray([rng.uniform(-0.5, 0.5) for _ in range(n)], np.float32)
        tm = np.asarray([1462826734 + 5 * i + rng.randint(0, 4) for i in range(n)], np.int64)
        acc = np.asarray([rng.choice([0, 5, 15, 50, 100000]) for _ in range(n)], np.int32)
        out.append(encode_request("veh-%d" % k, lat, lon, tm, acc))
    return out


def mutate(rng, b):
    s = b.decode()
    ops = [
        lambda s: s.replace('"lat":', '"lat" :', 1),                      # whitespace
        lambda s: s.replace('"accuracy":', '"speed":1,"accuracy":', 1),  # unknown key
        lambda s: s.replace('"lon":', '"lat":1.5,"lon":', 1),            # duplicate key
        lambda s: s.replace('"time":1', '"time":1.0e0+1', 1),            # exponent / junk
        lambda s: s.replace('"time":', '"time":"', 1),                    # string time
        lambda s: s.replace(',"accuracy":', ',"accuracy":-', 1),          # negative accuracy
        lambda s: s.replace('"uuid":"', '"uuid":"\\u00e9', 1),           # escape in uuid
        lambda s: s.replace('"uuid":"veh', '"uuid":null,"x":"veh', 1),    # null uuid + extra
        lambda s: s + " ",                                               # trailing space
        lambda s: s.replace('{"lat"', '{"accuracy":7,"time":3,"lat"', 1),  # reordered + duplicates
        lambda s: s[: s.index("},{") + 1] + "]}",                         # one point
        lambda s: s.replace('"lat":3', '"lat":03', 1),                    # leading zero
        lambda s: s.replace('"lat":3', '"lat":-0.0', 1),                  # negative zero
        lambda s: s.replace('"time":1', '"time":12345678901234567891', 1),  # bigint
        lambda s: '{"trace":' + s[s.index('"trace":') + 8:-1] + ',"uuid":"z"}',  # key order
        lambda s: s.replace(',"accuracy":', ',"accuracy":1.5,"x":', 1),
    ]
    return rng.choice(ops)(s).encode()


def test_fast_reader_matches_dom_on_java_bytes():
    rng = random.Random(5)
    for body in java_bodies(rng, 300):
        nf, f = points(body, True)
        nd, d = points(body, False)
        assert nf == nd and nf >= 2, body[:80]
        assert f == d, body[:80]


def test_fast_reader_rejects_or_agrees_on_variants():
    rng = random.Random(6)
    seen_reject = 0
    for body in java_bodies(rng, 150):
        for _ in range(6):
            v = mutate(rng, body)
            nf, f = points(v, True)
            nd, d = points(v, False)
            if nf == -2:
                seen_reject += 1
                continue
            assert nf >= 2 and nf == nd, v[:120]
            assert f == d, v[:120]
    assert seen_reject > 100


@pytest.mark.parametrize("body", [b"", b"{}", b"[]", b'{"uuid":"a","trace":[]}', b'{"uuid":"a"}',
                                  b'{"uuid":"a","trace":[{"lat":1,"lon":2,"time":3}]}',
                                  b'{"uuid":"a","trace":[{"lat":1,"lon":2,"time":3},{"lat":1,"lon":2}]}'])
def test_fast_reader_hands_back_invalid_requests(body):
    assert points(body, True)[0] == -2


def test_decimal_reading_is_correctly_rounded():
    """Float literals as float('...') reads them (json.loads), on both readers:
    the short-decimal fast path (<= 15 digits, one exact division) and the
    from_chars / strtod fallback for longer ones.  `time` keeps the double."""
    rng = random.Random(9)
    lits = ["0.1", "-0.0", "0.3", "1462826734.5", "123456789012345.6", "0.000000000000001",
            "9007199254740993.0", "1.7976931348623157", "2.2250738585072014", "1234567.000000001",
            "0.12345678901234567890123", "4.35", "100000000000000.0", "999999999999999.9"]
    for _ in range(3000):
        nd = rng.randint(1, 19)
        digits = "".join(rng.choice("0123456789") for _ in range(nd))
        cut = rng.randint(1, nd)
        ip = digits[:cut].lstrip("0") or "0"
        fp = digits[cut:] or "0"
        lits.append(("-" if rng.random() < 0.3 else "") + ip + "." + fp)
    for k in range(0, len(lits), 100):
        chunk = lits[k:k + 100]
        if len(chunk) < 2:
            chunk = chunk + ["0.5"]
        body = ('{"uuid":"u","trace":[' + ",".join('{"lat":37.5,"lon":-122.25,"time":%s}' % t for t in chunk)
                + "]}").encode()
        want = np.asarray([float(t) for t in chunk], np.float64).tobytes()
        for fast in (True, False):
            n, got = points(body, fast)
            assert n == len(chunk)
            assert got[2] == want, (fast, chunk)
