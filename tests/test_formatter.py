"""The native ingest formatter (otm_formatter, Formatter.java restated in C++)
against the reference's own documented examples and an independent Python
restatement (oracle/pyformatter.py) over a generated corpus of awkward
messages.  No JVM exists here: beyond the documented examples, parity is to
the Java library behaviour as restated."""
import itertools
import random

import numpy as np
import pytest

from reporter_amd.formatter import Formatter

README_SV = ",sv,\\|,1,9,10,0,5,yyyy-MM-dd HH:mm:ss"  # Reporter.java:38 / README.md:24
README_JSON = ",json,id,latitude,longitude,timestamp,accuracy"  # Reporter.java:42


def f32(x):
    return np.float32(x)


def test_reference_documented_examples():
    """Reporter.java:35-43 / README.md:23-27: the sv layout
    `time|uuid|x|x|x|accuracy|x|x|x|lat|lon|x|x|x` and the json object, with
    hand-computed expectations (2017-01-31 16:00:00 UTC = 1485878400)."""
    f = Formatter.GetFormatter(README_SV)
    key, (lat, lon, acc, t) = f.format("2017-01-31 16:00:00|uuid_abcdef|x|x|x|7.3|x|x|x|3.465725|-76.5135033|x|x|x")
    assert key == "uuid_abcdef" and t == 1485878400 and acc == 8
    assert lat == f32(3.465725) and lon == f32(-76.5135033)
    g = Formatter.GetFormatter(README_JSON)
    msg = '{"timestamp":1495037969,"id":"uuid_abcdef","accuracy":51.305,"latitude":3.465725,"longitude":-76.5135033}'
    key, (lat, lon, acc, t) = g.format(msg)
    assert key == "uuid_abcdef" and t == 1495037969 and acc == 52
    assert lat == f32(3.465725) and lon == f32(-76.5135033)
    # the README's @-separated spelling of the same json formatter (README.md:27)
    assert Formatter("@json@id@latitude@longitude@timestamp@accuracy").format(msg) == g.format(msg)


@pytest.mark.parametrize("text,want", [
    ("37.774929", 37.774929), ("-122.4194155", -122.4194155), (".5", 0.5), ("-.5", -0.5), ("5.", 5.0),
    ("007", 7.0), ("1,234.5", 1234.5), ("1,,2", 12.0), (",5", 5.0), ("12,", 12.0), ("1.5,3", 1.5),
    ("1E5", 1e5), ("2.5E-3", 2.5e-3), ("1E+5", 1.0), ("1e5", 1.0), ("1E", 1.0), ("5abc", 5.0),
    ("1.2.3", 1.2), ("-0", -0.0), ("0", 0.0), ("∞", np.inf), ("-∞", -np.inf),
    ("9223372036854775807", 9223372036854775807.0), ("-9223372036854775808", -9223372036854775808.0),
    ("16777217", 16777216.0), ("16777219", 16777220.0), ("1E4294967296", 1.0), ("0.1E-0", 0.1),
])
def test_decimal_format_parse_cases(text, want):
    """DecimalFormat("###.######").parse(..).floatValue() (JDK 8 semantics),
    expectations worked by hand from DecimalFormat.subparse / DigitList."""
    f = Formatter(",sv,\\|,0,1,2,3,4")
    key, (lat, lon, acc, t) = f.format("k|%s|0|0|0" % text)
    assert lat.tobytes() == f32(want).tobytes(), (text, lat, want)


@pytest.mark.parametrize("text", ["abc", "", "-", ".", "+5", " 5", "E5", ",", "-,"])
def test_decimal_format_parse_failures(text):
    f = Formatter(",sv,\\|,0,1,2,3,4")
    with pytest.raises(ValueError):
        f.format("k|%s|0|0|0" % text)


@pytest.mark.parametrize("spec", ["", ",xml,a,b", ",sv,\\|,1,2", ",json,a,b,c", ",sv,\\|,1,2,3,x,5",
                                  ",sv,(a|b),0,1,2,3,4", ",sv,a*,0,1,2,3,4", ",sv,\\|,0,1,2,3,4,yy-MM-dd",
                                  ",sv,\\|,0,1,2,3,4,EEE", ",json,a,b,c,d,e,MMM dd", "|sv|,|0|1|2|3|4"])
def test_spec_rejected(spec):
    """GetFormatter throws (bad type, too few args, NumberFormatException),
    or the spec is outside the supported subset -- loudly, at create."""
    with pytest.raises(ValueError):
        Formatter(spec)


# ---------------------------------------------------------------- corpus
NUMS = ["37.774929", "-122.4194155", "1,234.5", "1E5", "1E-5", "1E+5", "1e5", "5abc", "abc", "", ".5", "-.5",
        "-0", "007", "9223372036854775807", "9223372036854775808", "-9223372036854775808", "∞", "-∞", "�",
        "1.2.3", "12,", ",5", "1,,2", "  5", "+5", "1E99999999999", "0.000000001", "123456789012345678901234",
        "3.4028235E38", "3.5E38", "1.4E-45", "7E-46", "-1E-50", "0.30000000000000004", "١٢٣"]
EPOCHS = ["1485878400", "+1485878400", "-5", "12a", "", "9223372036854775807", "9223372036854775808", "0"]
DATES = ["2017-01-31 16:00:00", "2017-02-29 00:00:00", "2016-02-29 23:59:59", "2017-1-5 1:2:3",
         "99999-01-01 00:00:00", "-0001-03-01 00:00:00", "2017-01-31T16:00:00", "2017-01-31 16:00:00 ",
         "2017-13-01 00:00:00", "2017-01-31 24:00:00", "+2017-01-31 16:00:00", "1969-12-31 23:59:59",
         "2017-01-31 16:00:60", "1000000000-01-01 00:00:00", "2017-01-31 16:00"]
KEYS = ["uuid_abcdef", "", "ünïcødé-車", "a b", "k\x01"]


def random_numeric(rng):
    r = rng.random()
    if r < 0.5:
        return rng.choice(NUMS)
    v = rng.uniform(-200, 200) * 10 ** rng.randint(-8, 8)
    return rng.choice(["%r", "%.6f", "%.3e", "%.9g", "%.0f"]) % v


def sv_corpus(rng, n, sep, dated):
    msgs = []
    for _ in range(n):
        fields = [rng.choice(KEYS), random_numeric(rng), random_numeric(rng),
                  rng.choice(DATES) if dated else rng.choice(EPOCHS), random_numeric(rng)]
        if rng.random() < 0.05:
            fields = fields[:rng.randint(0, 4)]
        msg = sep.join(fields)
        if rng.random() < 0.05:
            msg += sep * rng.randint(1, 3)
        if rng.random() < 0.03:
            msg = msg.encode("utf-8") + b"\xff\xfe"
        elif rng.random() < 0.03:  # an encoded surrogate: one U+FFFD in JDK 8, three in Python's 'replace'
            msg = b"\xed\xa0\x80" + msg.encode("utf-8") + b"\xed\xa0"
        msgs.append(msg)
    return msgs


def json_value(rng, kind):
    r = rng.random()
    if kind == "num":
        if r < 0.4:
            return "%r" % rng.uniform(-180, 180)
        if r < 0.6:
            return '"%s"' % rng.choice(NUMS).replace('"', "")
        return rng.choice(["1", "-0", "1e5", "1.5E-7", "123456789012345678901234", "true", "null", "{}", "[1]",
                           '"  42 "', "0.1", "-1e400", "12345678"])
    if kind == "time":
        return rng.choice(["1495037969", '"1495037969"', '" +1495037969 "', '"1.5e9"', "1.5e9", '"0x1p3"',
                           '"NaN"', "true", "null", '"abc"', "99999999999999999999", "-1495037969.9", '"12f"'])
    if kind == "date":
        return '"%s"' % rng.choice(DATES) if r < 0.8 else rng.choice(["1495037969", "null"])
    if kind == "key":
        return rng.choice(['"uuid_abcdef"', '"\\u00fcn\\u00efc\\ud83d\\ude00"', '"\\ud800x\\udc00"', "12345", "1.5", "1e21", "true",
                           "null", "{}", '""', "1.0E-5", "100", "0.001"])
    raise ValueError(kind)


def json_corpus(rng, n, dated):
    msgs = []
    for _ in range(n):
        pairs = [("id", json_value(rng, "key")), ("latitude", json_value(rng, "num")),
                 ("longitude", json_value(rng, "num")), ("timestamp", json_value(rng, "date" if dated else "time")),
                 ("accuracy", json_value(rng, "num"))]
        rng.shuffle(pairs)
        if rng.random() < 0.05:
            pairs.pop(rng.randrange(len(pairs)))
        if rng.random() < 0.05:
            pairs.append(("latitude", json_value(rng, "num")))  # duplicate key: last wins
        msg = "{" + ",".join('"%s":%s' % kv for kv in pairs) + "}"
        r = rng.random()
        if r < 0.03:
            msg += " trailing garbage"
        elif r < 0.05:
            msg = "[" + msg + "]"
        elif r < 0.07:
            msg = msg.replace("}", ',"x":NaN}')
        elif r < 0.09:
            msg = msg[:-3]
        elif r < 0.11:
            msg = "  \n" + msg
        msgs.append(msg)
    return msgs


SPECS = [
    (",sv,\\|,1,9,10,0,5,yyyy-MM-dd HH:mm:ss", "readme"),
    ("@sv@,@0@1@2@3@4", "comma_epoch"),
    (";sv;\\s+;0;1;2;3;4", "whitespace_run"),
    (",sv,[;|],0,1,2,3,4,yyyy-MM-dd HH:mm:ss", "class_dated"),
    (",sv,\\t,0,1,2,3,4", "tab"),
    (",json,id,latitude,longitude,timestamp,accuracy", "json_epoch"),
    (",json,id,latitude,longitude,timestamp,accuracy,yyyy-MM-dd HH:mm:ss", "json_dated"),
]


def _layout(spec):
    if spec.startswith(",sv,\\|,1,9,10,0,5"):
        return "readme"
    return None


def make_corpus(spec, n, seed):
    rng = random.Random(seed)
    if ",json," in spec:
        return json_corpus(rng, n, dated=spec.count(",") > 6)
    if spec.startswith(",sv,\\|,1,9,10,0,5"):
        # the README layout: time|uuid|x|x|x|accuracy|x|x|x|lat|lon|x|x|x
        msgs = []
        for _ in range(n):
            f = ["x"] * 14
            f[0], f[1], f[5] = rng.choice(DATES), rng.choice(KEYS), random_numeric(rng)
            f[9], f[10] = random_numeric(rng), random_numeric(rng)
            msgs.append("|".join(f[:rng.choice([14, 14, 14, 9, 11])]))
        return msgs
    sep = {"@sv@,": ",", ";sv;\\s+": rng.choice([" ", "\t ", "  "]), ",sv,[;|]": rng.choice([";", "|"]),
           ",sv,\\t": "\t"}
    for prefix, s in sep.items():
        if spec.startswith(prefix):
            return sv_corpus(rng, n, s, dated="yyyy" in spec)
    raise ValueError(spec)


def _same(a, b):
    return a.tobytes() == b.tobytes() or (np.isnan(a) and np.isnan(b))


@pytest.mark.parametrize("spec", [s for s, _ in SPECS], ids=[i for _, i in SPECS])
def test_corpus_matches_restatement(spec):
    from oracle import pyformatter as P
    msgs = make_corpus(spec, 1500, seed=hash(spec) & 0xFFFF)
    got = Formatter(spec).format_many(msgs)
    ref = P.Formatter(spec)
    n_ok = 0
    for i, m in enumerate(msgs):
        try:
            want = ref.format(m)
        except P.Drop:
            want = None
        assert bool(got["ok"][i]) == (want is not None), (m, want)
        if want is None:
            continue
        n_ok += 1
        key, lat, lon, acc, t = want
        assert got["keys"][i] == key, m
        assert _same(got["lat"][i], lat) and _same(got["lon"][i], lon), (m, got["lat"][i], lat, got["lon"][i], lon)
        assert got["accuracy"][i] == acc and got["time"][i] == t, (m, got["accuracy"][i], acc, got["time"][i], t)
    # the corpus exercised both outcomes
    assert 0.1 * len(msgs) < n_ok < len(msgs)


def test_threads_do_not_change_results():
    spec = SPECS[0][0]
    msgs = make_corpus(spec, 40000, seed=3)
    f = Formatter(spec)
    a, b = f.format_many(msgs, nthreads=1), f.format_many(msgs, nthreads=6)
    for k in ("ok", "lat", "lon", "accuracy", "time"):
        assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), k
    assert a["keys"] == b["keys"]


def test_time_patterns():
    """joda patterns: fixed-width adjacent fields, fractions (truncated to
    millis), quoted literals, case-insensitive literals, default year 2000."""
    def t(pattern, text):
        f = Formatter("#sv#,#0#1#2#3#4#" + pattern)
        try:
            return f.format("k,1,1,%s,1" % text)[1][3]
        except ValueError:
            return None
    assert t("yyyyMMdd'T'HHmmss", "20170131T160000") == 1485878400
    assert t("yyyyMMdd'T'HHmmss", "20170131t160000") == 1485878400
    assert t("yyyy-MM-dd HH:mm:ss.SSS", "2017-01-31 16:00:00.999") == 1485878400
    assert t("yyyy-MM-dd HH:mm:ss.S", "1969-12-31 23:59:59.5") == 0  # -500 ms / 1000 truncates toward zero
    assert t("MM/dd HH", "02/29 01") == 951786000  # 2000-02-29 01:00 UTC
    assert t("HH:mm", "01:30") == 5400
    assert t("yyyy-MM-dd", "2017-02-29") is None
    assert t("yyyy-MM-dd''HH", "2017-01-31'16") == 1485878400
    assert t("yyyy", "-1") == -62198755200  # 0000 -> year -1, proleptic ISO


def test_batcher_process_raw_equals_formatted_records(small_graph, oracle):
    """The raw topology (formatter -> batcher) equals formatting first and
    feeding the formatted records; dropped messages are counted."""
    from reporter_amd.batcher import Batcher
    from test_batcher import make_stream
    recs = make_stream(small_graph, n_veh=12, n_pts=40, seed=45)
    msgs, ts = [], []
    for i, (key, lat, lon, acc, t) in enumerate(recs):
        msgs.append('{"id":"%s","latitude":%r,"longitude":%r,"timestamp":%d,"accuracy":%d}' % (key, lat, lon, t, acc))
        ts.append(t * 1000)
        if i % 50 == 7:
            msgs.append("not json")
            ts.append(t * 1000)
    g = oracle.Graph(small_graph)
    handler = lambda bodies: [oracle.handle_request(g, x) for x in bodies]  # noqa: E731
    fmt = Formatter(README_JSON)
    a = Batcher(handler=handler)
    a.process_raw(fmt, msgs, ts)
    a.close()
    fm = fmt.format_many(msgs)
    ok = fm["ok"]
    b = Batcher(handler=handler)
    b.process([k for k, o in zip(fm["keys"], ok) if o], fm["lat"][ok], fm["lon"][ok], fm["accuracy"][ok],
              fm["time"][ok], np.asarray(ts)[ok])
    b.close()
    sa, sb = a.stats(), b.stats()
    assert sa["raw_messages"] == len(msgs) and sa["raw_dropped"] == len(msgs) - len(recs)
    for k in ("records", "requests", "forwarded", "clean_ops", "stored_points"):
        assert sa[k] == sb[k], k
    assert sorted(a.forwarded()) == sorted(b.forwarded())
