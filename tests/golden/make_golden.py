#!/usr/bin/env python3
"""Generate golden fixtures from the REFERENCE itself (run in the build container only).

This is test infrastructure.  It imports the reference's own Python code from
/root/reference (read-only, never copied) behind in-memory shims and records
its input/output behaviour as JSON data under tests/golden/:

  report_cases.json   -- SegmentMatcherHandler.handle_request/report
                         (py/reporter_service.py:110-240) driven with canned
                         matcher outputs (a stub `valhalla` module), across the
                         REPORT_LEVELS / TRANSITION_LEVELS / THRESHOLD_SEC env
                         configurations read by make_thread_locals (:51-62).
  request_cases.json  -- the HTTP-level error contract of parse_trace /
                         handle_request (:85-106, :218-240) for malformed bodies.
  env_cases.json      -- make_thread_locals' env parsing quirks (:55-62).
  transport_cases.json -- the /report bytes of Java keys (uuids) outside
                         ASCII, as HttpClient.POST sends them (StringEntity's
                         ISO-8859-1, HttpClient.java:26; '?' above U+00FF), and
                         the reference's answer to those bytes
                         (body.decode('utf-8') at :99, then :218-240).
  decode_cases.json   -- generate_test_trace.decode (py/generate_test_trace.py:9-29)
  synth_cases.json    -- generate_test_trace.synthesize_gps (:31-73), stddev=0,
                         wall clock pinned.

Shims: Queue/BaseHTTPServer/SocketServer module
aliases, cgi.urlparse = urllib.parse, a stub `valhalla` module.  Bytecode
writing is disabled so nothing is written under /root/reference.
generate_test_trace.py is Python 2 (print statement at :88); it is converted
with lib2to3's fix_print IN MEMORY and exec'd.

Nothing in tests/ or the product imports this script or /root/reference at
run time; only the JSON it writes is committed.
"""
import sys
sys.dont_write_bytecode = True
import os
import io
import json
import random
import queue
import http.server
import socketserver
import urllib.parse
import importlib.util
import types
import warnings

warnings.simplefilter("ignore")
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# ---------------------------------------------------------------- shims
class _StubMatcher(object):
    canned = '{"segments":[]}'
    last_input = None

    def Match(self, s):
        _StubMatcher.last_input = s
        c = _StubMatcher.canned
        if isinstance(c, Exception):
            raise c
        return c


def _install_shims():
    sys.modules["Queue"] = queue
    sys.modules["BaseHTTPServer"] = http.server
    sys.modules["SocketServer"] = socketserver
    import cgi
    cgi.urlparse = urllib.parse
    v = types.ModuleType("valhalla")
    v.SegmentMatcher = _StubMatcher
    v.Configure = lambda path: None
    sys.modules["valhalla"] = v


def load_reporter_service():
    _install_shims()
    spec = importlib.util.spec_from_file_location(
        "ref_reporter_service", os.path.join(REF, "py/reporter_service.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def load_generate_test_trace():
    from lib2to3.refactor import RefactoringTool
    src = open(os.path.join(REF, "py/generate_test_trace.py")).read()
    tool = RefactoringTool(["lib2to3.fixes.fix_print"])
    py3 = str(tool.refactor_string(src, "generate_test_trace.py"))
    ns = {"__name__": "ref_generate_test_trace"}
    exec(compile(py3, "generate_test_trace.py", "exec"), ns)
    return ns


# ---------------------------------------------------------------- helpers
ENV_KEYS = ("REPORT_LEVELS", "TRANSITION_LEVELS", "THRESHOLD_SEC")


def set_env(env):
    for k in ENV_KEYS:
        os.environ.pop(k, None)
    for k, v in env.items():
        os.environ[k] = v


class _FakeHeaders(dict):
    pass


def run_handler(mod, body_bytes, path="/report", post=True):
    """Drive SegmentMatcherHandler.do()'s logic without sockets: returns
    (code, body) exactly as answer() would receive them."""
    h = mod.SegmentMatcherHandler.__new__(mod.SegmentMatcherHandler)
    h.path = path
    h.headers = _FakeHeaders({"Content-Length": str(len(body_bytes))})
    h.rfile = io.BytesIO(body_bytes)
    err = io.StringIO()
    old = sys.stderr
    sys.stderr = err
    try:
        try:
            code, body = h.handle_request(post)
        except Exception as e:  # do(): answer(400, str(e))
            code, body = 400, str(e)
    finally:
        sys.stderr = old
    return code, body, err.getvalue()


def init_thread_locals(mod):
    tp = mod.ThreadPoolMixIn.__new__(mod.ThreadPoolMixIn)
    tp.make_thread_locals()


# ---------------------------------------------------------------- report cases
def mk_trace(n, t0=1000, dt=10, float_time=False, uuid="abc"):
    pts = []
    for i in range(n):
        t = t0 + dt * i
        pts.append({"lat": round(14.5 + 0.0003 * i, 6), "lon": round(121.0 + 0.0004 * i, 6),
                    "time": float(t) if float_time else t, "accuracy": 5})
    return {"uuid": uuid, "trace": pts}


def seg(sid=None, st=-1, et=-1, length=-1, internal=False, b=0, e=0, ways=(1,), ql=0):
    d = {}
    if sid is not None:
        d["segment_id"] = sid
    d["way_ids"] = list(ways)
    d["start_time"] = st
    d["end_time"] = et
    d["queue_length"] = ql
    d["length"] = length
    d["internal"] = internal
    d["begin_shape_index"] = b
    d["end_shape_index"] = e
    return d


def appendix_c_cases():
    """SURVEY.md Appendix C probe cases (13 points, time = 1000 + 10 i)."""
    c = {}
    c["B"] = [seg((1 << 3) | 0, 1000.0, 1100.0, 500, b=0, e=5),
              seg((2 << 3) | 0, 1100.0, 1120.0, 400, b=5, e=12)]
    c["C"] = [seg((1 << 3) | 1, -1, 1030.0, -1, b=0, e=3),
              seg((2 << 3) | 1, 1030.0, 1060.0, 300, b=3, e=6),
              seg((3 << 3) | 1, -1, 1080.0, -1, b=6, e=8),
              seg((4 << 3) | 1, 1080.0, 1100.0, 200, b=8, e=10),
              seg((5 << 3) | 1, 1100.0, 1120.0, 200, b=10, e=12)]
    c["D"] = [seg((1 << 3) | 0, 1000.0, 1000.0, 500, b=0, e=5),
              seg((2 << 3) | 0, 1000.0, 1110.0, 400, b=5, e=12)]
    c["E"] = [seg((1 << 3) | 2, 1000.0, 1020.0, 150, b=0, e=2),
              seg(None, 1020.0, 1022.0, -1, internal=True, b=2, e=2),
              seg((3 << 3) | 1, 1022.0, 1050.0, 300, b=2, e=5),
              seg(None, 1050.0, 1060.0, -1, b=5, e=6),
              seg((5 << 3) | 0, 1060.0, 1090.0, 600, b=6, e=9),
              seg((6 << 3) | 0, 1090.0, 1115.0, 600, b=9, e=12)]
    c["F"] = []
    c["G"] = [seg((1 << 3) | 0, 1000.0, 1010.0, 1000, b=0, e=1),
              seg((2 << 3) | 0, 1010.0, 1100.0, 500, b=1, e=10),
              seg((3 << 3) | 0, 1100.0, 1120.0, 300, b=10, e=12)]
    c["H"] = [seg(None, 1000.0, 1005.0, -1, internal=True, b=0, e=1),
              seg((2 << 3) | 0, 1005.0, -1, -1, b=1, e=4),
              seg((3 << 3) | 0, -1, 1070.0, -1, b=4, e=7),
              seg((4 << 3) | 0, 1070.0, 1110.0, 400, b=7, e=11),
              seg((5 << 3) | 0, 1110.0, 1120.0, 100, b=11, e=12)]
    c["I"] = [seg((1 << 3) | 1, 1000.0, 1040.0, 400, b=0, e=4),
              seg((2 << 3) | 0, 1040.0, 1070.0, 300, b=4, e=7),
              seg((3 << 3) | 1, 1070.0, 1100.0, 300, b=7, e=10),
              seg((4 << 3) | 0, 1100.0, 1120.0, 200, b=10, e=12)]
    return c


def random_segments(rng, n_pts, t0):
    """A random but plausible Match output for an n_pts trace."""
    segs = []
    n = rng.randint(0, 9)
    t = float(t0) + rng.choice([0.0, rng.uniform(0, 20)])
    idx = 0
    prev_end_partial = False
    for k in range(n):
        kind = rng.random()
        internal = kind < 0.12
        has_id = (not internal) and rng.random() > 0.15
        level = rng.choice([0, 0, 1, 1, 2])
        sid = None
        if has_id:
            sid = (rng.randint(1, 1 << 40) << 3) | level
            if rng.random() < 0.1:
                sid = (rng.randint(1 << 55, (1 << 60)) << 3) | level
        dur = rng.choice([rng.uniform(0.5, 90.0), float(rng.randint(1, 60))])
        if rng.random() < 0.03:
            dur = 0.0
        length = rng.choice([rng.randint(20, 1000), rng.randint(20, 1000), -1])
        if rng.random() < 0.08:
            length = rng.randint(1500, 4000)  # often too fast -> invalid speed
        st = round(t, rng.choice([0, 1, 3, 6, 9]))
        et = round(t + dur, rng.choice([0, 1, 3, 6, 9]))
        if rng.random() < 0.2 or (prev_end_partial and rng.random() < 0.5):
            st = -1
            length = -1
        if rng.random() < 0.2:
            et = -1
            length = -1
        if rng.random() < 0.1 and st != -1:
            st = int(st)
        prev_end_partial = et == -1
        b = min(idx, n_pts - 1)
        idx = min(n_pts - 1, idx + rng.randint(0, 3))
        ways = [rng.randint(1, 10 ** 9) for _ in range(rng.randint(0, 3))]
        segs.append(seg(sid, st, et, length, internal, b, idx, ways, ql=rng.choice([0, 0, 0, 12])))
        t = t + dur
    return segs


ENV_CONFIGS = [
    {},
    {"REPORT_LEVELS": "0", "TRANSITION_LEVELS": "0"},
    {"REPORT_LEVELS": "0,1,2", "TRANSITION_LEVELS": "0,1,2"},
    {"REPORT_LEVELS": "1", "TRANSITION_LEVELS": "0,1,2"},
    {"THRESHOLD_SEC": "true"},
    {"THRESHOLD_SEC": "false"},
    {"THRESHOLD_SEC": ""},
    {"REPORT_LEVELS": " 0, 2", "TRANSITION_LEVELS": "2", "THRESHOLD_SEC": "Off"},
]


def make_report_cases(mod):
    rng = random.Random(20171015)
    cases = []
    for env in ENV_CONFIGS:
        set_env(env)
        init_thread_locals(mod)
        for name, segs in appendix_c_cases().items():
            trace = mk_trace(13)
            cases.append(run_report_case(mod, "appC_" + name, env, trace,
                                         json.dumps({"segments": segs}, separators=(",", ":"))))
        for k in range(60):
            n = rng.randint(2, 40)
            trace = mk_trace(n, t0=rng.choice([1000, 1500000000]), dt=rng.choice([1, 5, 10, 30]),
                             float_time=rng.random() < 0.2, uuid=rng.choice(["u1", "999999", 42]))
            segs = random_segments(rng, n, trace["trace"][0]["time"])
            canned = json.dumps({"segments": segs}, separators=(",", ":"))
            if rng.random() < 0.1:  # non-canonical matcher output formatting
                canned = json.dumps({"segments": segs}, indent=1).replace("1.0,", "1.00,")
            cases.append(run_report_case(mod, "rand%d" % k, env, trace, canned))
    # matcher output with extra keys / passthrough oddities
    set_env({})
    init_thread_locals(mod)
    trace = mk_trace(5)
    odd = ('{"segments":[{"segment_id":9,"way_ids":[],"start_time":1000,"end_time":1010.5,'
           '"queue_length":0,"length":80,"internal":false,"begin_shape_index":0,"end_shape_index":2,'
           '"extra":{"u":"caf\\u00e9","e":1E3,"f":1.50,"n":null}},'
           '{"segment_id":17,"start_time":1010.5,"end_time":1040.25,"length":300,'
           '"begin_shape_index":2,"end_shape_index":4}],"mode":"bike","zz":[1,2.5e-7,1e16,123456789012.0]}')
    cases.append(run_report_case(mod, "passthrough", {}, trace, odd))
    cases.append(run_report_case(mod, "match_raises", {}, trace, RuntimeError("boom")))
    # time missing on last point -> KeyError inside report -> 500
    t2 = mk_trace(4)
    del t2["trace"][-1]["time"]
    cases.append(run_report_case(mod, "last_point_no_time", {}, t2, '{"segments":[]}'))
    return cases


def run_report_case(mod, name, env, trace, canned):
    _StubMatcher.canned = canned
    _StubMatcher.last_input = None
    body = json.dumps(trace).encode("utf-8")
    code, resp, err = run_handler(mod, body)
    return {"name": name, "env": env, "request": body.decode("utf-8"),
            "match_output": canned if isinstance(canned, str) else None,
            "match_error": str(canned) if isinstance(canned, Exception) else None,
            "match_input": _StubMatcher.last_input, "code": code, "body": resp,
            "stderr": err}


# ---------------------------------------------------------------- request cases
def make_request_cases(mod):
    set_env({})
    init_thread_locals(mod)
    _StubMatcher.canned = '{"segments":[]}'
    bodies = [
        b"", b" ", b"{", b"[1,2", b'{"uuid":1,}', b"nul", b"{'a':1}", b'{"a" 1}', b'{"a":1 "b":2}',
        b'{"a":"x\x01"}', b'{"a":"\\q"}', b'{"a":1}x', b'\n\n  {"a":tru}', b'{"a":"\xc3\xa9\\u00e9",]}',
        b"[]", b"[1]", b'"str"', b"12", b"1.5", b"true", b"null",
        b"{}", b'{"uuid":null,"trace":[]}', b'{"uuid":"a"}', b'{"uuid":"a","trace":[]}',
        b'{"uuid":"a","trace":[{"lat":1,"lon":2,"time":3}]}', b'{"uuid":"a","trace":{}}',
        b'{"uuid":"a","trace":{"1":2}}', b'{"uuid":"a","trace":"x"}', b'{"uuid":"a","trace":5}',
        b'{"uuid":"a","trace":null}', b'{"uuid":"a","trace":true}',
        b'{"uuid":0,"trace":[{"lat":1,"lon":2,"time":3},{"lat":1,"lon":2,"time":4}]}',
        b'{"uuid":"","trace":[{"lat":1,"lon":2,"time":3},{"lat":1,"lon":2,"time":4}]}',
        b'{"uuid":"a","uuid":null,"trace":[1,2]}',
    ]
    cases = []
    for b in bodies:
        code, resp, err = run_handler(mod, b)
        cases.append({"body": b.decode("utf-8", "surrogateescape"), "body_hex": b.hex(), "code": code,
                      "response": resp, "match_input": _StubMatcher.last_input})
        _StubMatcher.last_input = None
    # action routing (parse_trace :92-96)
    for path in ["/report", "/report?x=1", "/foo", "/", "/a/b/report"]:
        code, resp, err = run_handler(mod, b'{"uuid":"a","trace":[]}', path=path)
        cases.append({"path": path, "body": '{"uuid":"a","trace":[]}', "code": code, "response": resp})
    return cases


def make_env_cases(mod):
    out = []
    for env in ENV_CONFIGS + [{"THRESHOLD_SEC": "15"}, {"THRESHOLD_SEC": "yes"}, {"REPORT_LEVELS": ""},
                              {"TRANSITION_LEVELS": "1,x"}, {"REPORT_LEVELS": "+1,-2, 3 "}]:
        set_env(env)
        rec = {"env": env}
        try:
            init_thread_locals(mod)
            tl = mod.thread_local
            rec["report_levels"] = sorted(tl.report_levels)
            rec["transition_levels"] = sorted(tl.transition_levels)
            rec["threshold_sec"] = tl.threshold_sec
            rec["threshold_type"] = type(tl.threshold_sec).__name__
        except Exception as e:
            rec["error"] = "%s: %s" % (type(e).__name__, e)
        out.append(rec)
    set_env({})
    return out


# ---------------------------------------------------------------- transport (HttpClient charsets)
# (coordinates exact in float32, so the Java batcher writes exactly this text)
TRANSPORT_TRACE = ('{"lat":14.5,"lon":121.25,"time":1000,"accuracy":5},'
                   '{"lat":14.5,"lon":121.5,"time":1010,"accuracy":5}')
# Java Strings as UTF-16 code units (a lone surrogate included)
TRANSPORT_KEYS = [
    ("latin1_e_acute", [0xE9]),
    ("latin1_two", [0x61, 0xE9, 0xE8]),
    ("latin1_y_diaeresis", [0xFF]),
    ("latin1_trailing_lead_byte", [0x78, 0xC3]),
    ("latin1_pair_forms_utf8", [0xC3, 0xA9]),            # "Ã©" -> C3 A9 = UTF-8 for U+00E9
    ("latin1_four_forms_utf8", [0xF0, 0x9F, 0x98, 0x80]),  # -> F0 9F 98 80 = UTF-8 for U+1F600
    ("latin1_forms_surrogate", [0xED, 0xA0, 0x80]),      # -> ED A0 80: Python rejects surrogates
    ("latin1_nbsp", [0xA0]),
    ("cjk", [0x65E5, 0x672C]),                           # -> "??"
    ("supplementary", [0x61, 0xD83D, 0xDE00, 0x62]),     # a surrogate pair -> one '?'
    ("lone_high_surrogate", [0xD800, 0x61]),
    ("lone_low_surrogate", [0x61, 0xDC00]),
    ("replacement_char", [0xFFFD]),
    ("mixed", [0x75, 0x2D, 0x65E5, 0xE9]),
    ("quote", [0x61, 0x22, 0x62]),                        # sb.append(key) is unescaped (Batch.java:55)
    ("backslash", [0x61, 0x5C, 0x62]),
    ("backslash_u", [0x5C, 0x75, 0x30, 0x30, 0x65, 0x39]),
    ("control", [0x61, 0x01]),
    ("delete", [0x7F]),
    ("ascii", [0x76, 0x65, 0x68, 0x30, 0x31]),
]


def java_latin1(units):
    """String.getBytes(ISO_8859_1) on UTF-16 code units (JDK 8 REPLACE): a
    unit above U+00FF becomes '?', a high+low surrogate pair one '?'."""
    out = bytearray()
    i = 0
    while i < len(units):
        u = units[i]
        if u <= 0xFF:
            out.append(u)
        else:
            if 0xD800 <= u <= 0xDBFF and i + 1 < len(units) and 0xDC00 <= units[i + 1] <= 0xDFFF:
                i += 1
            out.append(0x3F)
        i += 1
    return bytes(out)


def java_utf8(units):
    """String.getBytes(UTF_8) (Kafka's StringSerializer): the record key's
    bytes on the formatted topic; an unpaired surrogate becomes '?'."""
    out = bytearray()
    i = 0
    while i < len(units):
        u = units[i]
        if 0xD800 <= u <= 0xDBFF and i + 1 < len(units) and 0xDC00 <= units[i + 1] <= 0xDFFF:
            out += chr(0x10000 + ((u - 0xD800) << 10) + (units[i + 1] - 0xDC00)).encode("utf-8")
            i += 2
            continue
        out += b"?" if 0xD800 <= u <= 0xDFFF else chr(u).encode("utf-8")
        i += 1
    return bytes(out)


def make_transport_cases(mod):
    set_env({})
    init_thread_locals(mod)
    _StubMatcher.canned = '{"segments":[]}'
    cases = []
    for name, units in TRANSPORT_KEYS:
        key_wire = java_latin1(units)
        body = b'{"uuid":"' + key_wire + b'","trace":[' + TRANSPORT_TRACE.encode() + b"]}"
        _StubMatcher.last_input = None
        code, resp, err = run_handler(mod, body)
        cases.append({"name": name, "key_utf16": units, "key_utf8_hex": java_utf8(units).hex(),
                      "body_hex": body.hex(), "code": code, "response": resp,
                      "match_input": _StubMatcher.last_input})
    return cases


# ---------------------------------------------------------------- decode / synthesize_gps
def encode_polyline6(coords_lonlat):
    """Test-side encoder (Google polyline algorithm, precision 1e6) used only
    to manufacture inputs for the reference decoder."""
    out = []
    prev = [0, 0]
    for lon, lat in coords_lonlat:
        for j, v in enumerate((int(round(lat * 1e6)), int(round(lon * 1e6)))):
            d = v - prev[j]
            prev[j] = v
            d = ~(d << 1) if d < 0 else (d << 1)
            while d >= 0x20:
                out.append(chr((0x20 | (d & 0x1f)) + 63))
                d >>= 5
            out.append(chr(d + 63))
    return "".join(out)


def make_decode_cases(gtt):
    rng = random.Random(7)
    cases = [{"encoded": "_izlhA~rlgdF_{geC~ywl@_kwzCn`{nI"}]
    for k in range(40):
        n = rng.randint(1, 30)
        lon0, lat0 = rng.uniform(-179, 179), rng.uniform(-85, 85)
        pts = [(lon0 + rng.uniform(-0.01, 0.01) * i, lat0 + rng.uniform(-0.01, 0.01) * i) for i in range(n)]
        cases.append({"encoded": encode_polyline6(pts)})
    cases.append({"encoded": ""})
    for c in cases:
        c["decoded"] = gtt["decode"](c["encoded"])
    return cases


def make_synth_cases(gtt):
    class _T:
        @staticmethod
        def time():
            return 1500086400.25
    gtt["t"] = _T
    rng = random.Random(11)
    cases = []
    for k in range(20):
        n = rng.randint(3, 25)
        lon0, lat0 = 23.7 + rng.uniform(-0.05, 0.05), 37.98 + rng.uniform(-0.05, 0.05)
        pts = [(lon0 + 0.0007 * i + rng.uniform(-1e-4, 1e-4), lat0 + 0.0005 * i) for i in range(n)]
        shape = encode_polyline6(pts)
        edges = []
        i = 0
        while i < n - 1:
            j = min(n - 1, i + rng.randint(1, 3))
            edges.append({"length": round(rng.uniform(0.02, 0.4), 3), "speed": rng.choice([20, 30, 45, 60, 90]),
                          "begin_shape_index": i, "end_shape_index": j})
            i = j
        res = gtt["synthesize_gps"](edges, shape, uuid="synth%d" % k)
        cases.append({"edges": edges, "shape": shape, "uuid": "synth%d" % k, "now": 1500086400.25,
                      "result": res})
    # out-of-range shape index -> (None, None)
    bad = gtt["synthesize_gps"]([{"length": 0.1, "speed": 30, "begin_shape_index": 0,
                                   "end_shape_index": 5}], encode_polyline6([(1, 2), (1.001, 2.001)]))
    cases.append({"edges": [{"length": 0.1, "speed": 30, "begin_shape_index": 0, "end_shape_index": 5}],
                  "shape": encode_polyline6([(1, 2), (1.001, 2.001)]), "uuid": "999999",
                  "now": 1500086400.25, "result": list(bad)})
    return cases


def dump(name, obj):
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=False)
        f.write("\n")


def main():
    mod = load_reporter_service()
    dump("report_cases.json", make_report_cases(mod))
    dump("request_cases.json", make_request_cases(mod))
    dump("env_cases.json", make_env_cases(mod))
    dump("transport_cases.json", make_transport_cases(mod))
    gtt = load_generate_test_trace()
    dump("decode_cases.json", make_decode_cases(gtt))
    dump("synth_cases.json", make_synth_cases(gtt))
    set_env({})
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
