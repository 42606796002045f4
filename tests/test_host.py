"""Host-side checks that need no GPU: the C ABI surface, the Java request
encoder, sharding, synthetic inputs and the oracle's own invariants."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from reporter_amd import _lib, encode_request, murmur2_partition, synth, tracegen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "otmatch.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(otm_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    for fn in header_functions():
        assert fn in exported, "%s declared in include/otmatch.h but not exported" % fn
        assert getattr(L, fn) is not None
    # and the binding declares a signature for each
    assert set(header_functions()) == set(_lib.EXPORTED)


def test_integration_sources_bind_exported_symbols():
    """The Java FFM / JNI sources under integration/ (not compiled here: no
    JDK) bind only functions include/otmatch.h declares and the library
    exports."""
    import glob
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    declared = set(header_functions())
    used = set()
    for f in glob.glob(os.path.join(root, "integration", "**", "*.*"), recursive=True):
        used |= set(re.findall(r"\b(otm_[a-z0-9_]+)\s*\(", open(f).read()))
        used |= set(re.findall(r'"(otm_[a-z0-9_]+)"', open(f).read()))
    assert {"otm_engine_create", "otm_report", "otm_submit", "otm_poll", "otm_free"} <= used
    assert used <= declared, used - declared


def test_library_is_gfx950_code():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data  # the offload bundle's code object entry


def test_engine_create_fails_loudly_without_gpu_or_bad_config(tmp_path):
    from reporter_amd import Engine, OtmError
    cfg = tmp_path / "c.json"
    cfg.write_text('{"otm":{}}')
    with pytest.raises(OtmError):
        Engine(config_path=str(cfg))


def test_encode_request_java_format():
    # Batch.java:52-61 + Point.java:39-45 (DecimalFormat "###.######", HALF_EVEN on the float value)
    b = encode_request("u1", [37.98, -0.5, 0.0, 1.0000005, 14.543087], [23.72, 0.25, -0.0, 100.0, 121.021019],
                       [1500000000, 1, 2, 3, 4], [15, 5, 0, 1, 9])
    assert b == (b'{"uuid":"u1","trace":[{"lat":37.98,"lon":23.719999,"time":1500000000,"accuracy":15},'
                 b'{"lat":-.5,"lon":.25,"time":1,"accuracy":5},{"lat":0,"lon":-0,"time":2,"accuracy":0},'
                 b'{"lat":1,"lon":100,"time":3,"accuracy":1},{"lat":14.543087,"lon":121.021019,"time":4,'
                 b'"accuracy":9}]}')
    # the service's parser accepts the ordinary case; the "-.5" quirk of "###" is kept on purpose
    assert encode_request("k", [], [], [], []) == b'{"uuid":"k","trace":]}'


def test_murmur2_sharding_is_kafka_partitioner():
    # Kafka Utils.murmur2 known answers (kafka-clients test vectors)
    L = _lib.lib()
    vec = {b"21": -973932308, b"foobar": -790332482, b"a-little-bit-long-string": -985981536,
           b"a-little-bit-longer-string": -1486304829,
           b"lkjh234lh9fiuh90y23oiuhsafujhadof229phr9h19h89h8": -58897971, b"abc": 479470107}
    for k, v in vec.items():
        assert L.otm_murmur2(k, len(k)) == v, k
    ids0 = synth.shard_vehicle_ids(500, 0, 4)
    ids1 = synth.shard_vehicle_ids(500, 1, 4)
    assert not set(ids0.tolist()) & set(ids1.tolist())
    assert all(murmur2_partition("veh%d" % v, 4) == 0 for v in ids0[:50])


def test_synthetic_inputs_deterministic(small_graph):
    a = synth.make_traces(small_graph, 20, 30, seed=5)
    b = synth.make_traces(small_graph, 20, 30, seed=5)
    for k in a:
        assert np.array_equal(a[k], b[k])
    # a vehicle depends only on its global id
    c = synth.make_traces(small_graph, 1, 30, seed=5, vehicle_ids=[7])
    assert np.array_equal(c["lat"], a["lat"][7 * 30:8 * 30])


def test_oracle_loads_graph_and_matches(small_graph, oracle):
    g = oracle.Graph(small_graph)
    b = synth.make_traces(small_graph, 50, 80, seed=2)
    r1 = oracle.match_batch(g, b, nthreads=1, keep_stages=True)
    r4 = oracle.match_batch(g, b, nthreads=4)
    for k in ("traces", "segments", "reports", "way_ids"):
        assert r1[k].tobytes() == r4[k].tobytes(), k
    st = r1["state"]
    ok = st >= 0
    assert ok.mean() > 0.95
    edges = r1["cand_edge"].reshape(-1, 32)[np.arange(len(st)), np.maximum(st, 0)]
    assert (edges[ok] == b["true_edge"][ok]).mean() > 0.8  # matched to the true directed edge
    c = r1["counters"]
    assert c["points"] == len(b["lat"]) and c["searches"] > 0 and c["nodes_settled"] >= c["searches"]


def test_oracle_node_candidates(small_graph, oracle):
    # node snap: a node candidate sits at offset 0 on its node's
    # first outgoing edge, one per node per point; candidates come in
    # distance order
    import struct
    raw = np.fromfile(small_graph, dtype=np.uint8)
    hs = struct.calcsize("<8sII4i2iq3d4dQ")

    def sec(i, dt):
        o, n = struct.unpack_from("<QQ", raw, hs + 16 * i)
        return np.frombuffer(raw, dtype=dt, count=n // np.dtype(dt).itemsize, offset=o)
    out_off, efrom = sec(2, np.int32), sec(3, np.int32)
    b = synth.make_traces(small_graph, 40, 80, seed=5)
    r = oracle.match_batch(oracle.Graph(small_graph), b, keep_stages=True)
    P = len(b["lat"])
    k = r["ncand"]
    e = r["cand_edge"].reshape(P, 32)
    o = r["cand_off"].reshape(P, 32)
    q = r["cand_emis"].reshape(P, 32)
    n_node = 0
    for p in range(P):
        ee, oo, qq = e[p, :k[p]], o[p, :k[p]], q[p, :k[p]]
        nd = ee[oo == 0.0]
        n_node += len(nd)
        assert len(np.unique(nd)) == len(nd)
        assert np.array_equal(nd, out_off[efrom[nd]])
        assert np.all(np.diff(qq) >= 0)  # (sqdist order; emission = sqdist / 2 sigma^2 can merge ulps)
    assert n_node > 0.05 * k.sum()


def test_oracle_json_path_config1(small_graph, oracle):
    """Config 1 plumbing: synthesize_gps traces -> handle_request -> 200s."""
    g = oracle.Graph(small_graph)
    bodies = tracegen.config1_requests(small_graph, n_traces=10, edges_per_trace=20)
    for body in bodies:
        code, resp = oracle.handle_request(g, body)
        assert code == 200, resp
        assert resp.startswith('{"stats":{"successful_matches":{"count":')


def test_cos_deg_accuracy(oracle):
    for d in np.linspace(-89.9, 89.9, 41):
        assert abs(oracle.cos_deg(float(d)) - np.cos(np.radians(d))) < 2e-7


def test_turn_cost_table():
    """meili's turn penalty table (turn_penalty_factor * exp(-theta / 45),
    theta the angle between the reversed incoming and the outgoing edge) in
    the oracle's 1/64 m units: straight on (deviation 0, theta 180) is the
    smallest penalty, a U-turn (deviation 180, theta 0) the whole factor."""
    import math
    from oracle import pyoracle
    L = pyoracle.lib()
    L.orc_turn_units.restype = C.c_uint32
    L.orc_turn_units.argtypes = [C.c_float, C.c_int]
    t = [L.orc_turn_units(200.0, d) for d in range(181)]
    assert t[180] == 200 * 64 and t[0] == round(200 * math.exp(-4) * 64)
    assert all(t[d] <= t[d + 1] for d in range(180))
    for d in (0, 45, 90, 135, 180):
        assert abs(t[d] - 200 * 64 * math.exp(-(180 - d) / 45.0)) <= 0.5
    assert all(L.orc_turn_units(0.0, d) == 0 for d in range(181))


def test_engine_create_device_arguments():
    """otm_engine_create's device list (no GPU needed: rejected before any
    device call): ndev < 1 or a NULL list is OTM_EINVAL; a NULL engine has
    no members."""
    L = _lib.lib()
    h = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    assert L.otm_engine_create(b"/nonexistent.json", devs, 0, C.byref(h)) == -1  # OTM_EINVAL
    assert L.otm_engine_create(b"/nonexistent.json", None, 2, C.byref(h)) == -1  # OTM_EINVAL
    assert not h.value
    assert L.otm_engine_members(None) == 0
    assert not L.otm_engine_member(None, 0)
    # a group whose members cannot be created fails as the member does
    assert L.otm_engine_create(b"/nonexistent.json", devs, 2, C.byref(h)) == -1  # OTM_EINVAL
    assert "cannot read config" in _lib.last_error()


def test_meili_config_mode_section_over_default(tmp_path):
    """meili's config layering: "default" with the mode's section on top.  A
    stock valhalla_build_config meili block has
    default.turn_penalty_factor 0 and auto.turn_penalty_factor 200: an auto
    match runs with 200 (no device needed: otm_config_meili)."""
    import json
    L = _lib.lib()
    cfg = tmp_path / "valhalla.json"

    def read(meili):
        cfg.write_text(json.dumps({"otm": {"graph": "g.otmg"}, "meili": meili}))
        p = _lib.MeiliParams()
        assert L.otm_config_meili(str(cfg).encode(), C.byref(p)) == 0, _lib.last_error()
        return p

    stock = {"mode": "auto", "customizable": ["mode", "search_radius"],
             "default": {"sigma_z": 4.07, "gps_accuracy": 5.0, "beta": 3, "max_route_distance_factor": 5,
                         "breakage_distance": 2000, "interpolation_distance": 10, "search_radius": 50,
                         "max_search_radius": 100, "turn_penalty_factor": 0},
             "auto": {"turn_penalty_factor": 200, "search_radius": 50},
             "pedestrian": {"turn_penalty_factor": 100, "search_radius": 25}}
    p = read(stock)
    assert p.turn_penalty_factor == 200.0 and p.search_radius == 50.0 and p.sigma_z == pytest.approx(4.07)
    # another mode's section applies instead
    p = read(dict(stock, mode="pedestrian"))
    assert p.turn_penalty_factor == 100.0 and p.search_radius == 25.0
    # no mode section: the default section alone
    p = read({"default": {"turn_penalty_factor": 0, "beta": 4}})
    assert p.turn_penalty_factor == 0.0 and p.beta == 4.0
    # no meili block at all: the built-in defaults (the auto costing's 200)
    p = read({})
    assert p.turn_penalty_factor == 200.0 and p.max_candidates == 32
    cfg.write_text(json.dumps({"meili": {"default": {"max_candidates": 99}}}))
    assert L.otm_config_meili(str(cfg).encode(), C.byref(p)) == -1
    assert "max_candidates" in _lib.last_error()


def test_null_engine_request_calls_fail_cleanly():
    """A NULL engine is a bad-arguments error on every request entry point,
    not a crash."""
    L = _lib.lib()
    out = C.c_void_p()
    n = C.c_size_t()
    body = b'{"uuid":"a","trace":[]}'
    assert L.otm_report(None, body, len(body), C.byref(out), C.byref(n)) < 0
    assert L.otm_match_json(None, body, len(body), C.byref(out), C.byref(n)) < 0


def test_arena_free_under_contention():
    """otm_free's lock-free arena scan while other threads release arenas and
    free plain pointers: every arena is released by its last body
    and no plain pointer is taken for an arena body (this also runs under
    TSan in tests/test_sanitizers.py)."""
    from reporter_amd._lib import lib
    assert lib().otm_debug_arena_stress(8, 200) == 0
    assert lib().otm_debug_arena_stress(3, 50) == 0
    assert lib().otm_debug_arena_stress(0, 1) == -1


def test_request_arena_release_contract():
    """otm_request_arena_release: NULL is a no-op, a pointer that is not an
    arena is refused; otm_request_arena_alloc either gives page-locked memory
    (a GPU box) or NULL with a message (no device here)."""
    import ctypes as C
    from reporter_amd._lib import last_error, lib
    L = lib()
    assert L.otm_request_arena_release(None) == 0
    buf = C.create_string_buffer(64)
    assert L.otm_request_arena_release(C.cast(buf, C.c_void_p)) < 0
    p = L.otm_request_arena_alloc(1 << 16)
    if p:
        C.memset(p, 0x41, 1 << 16)
        assert L.otm_request_arena_release(p) == 0
        assert L.otm_request_arena_release(p) < 0  # (released once)
    else:
        assert "page-locked" in last_error()
