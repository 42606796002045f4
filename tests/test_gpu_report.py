"""report() on the GPU (k_report) against the reference's own recorded outputs,
and the /report path under every env configuration the golden cases hold.

* The golden report cases (tests/golden/report_cases.json, recorded by
  running py/reporter_service.py itself behind a stub matcher) are fed
  straight to the kernel through otm_report_segments_device: their canned
  Match outputs become the kernel's segment records, and the response it
  builds must be the reference's (status, body, stderr) byte for byte, under
  each REPORT_LEVELS / TRANSITION_LEVELS / THRESHOLD_SEC configuration
  (make_thread_locals, py/reporter_service.py:51-62).
* Matched traces under the same env configurations: k_report after the GPU
  matcher, field by field against the oracle with the same report config.
* Config 1 (py/generate_test_trace.py's synthesize_gps traces) through
  otm_report_batch, byte-equal to the oracle's /report.
* The per-segment speed histogram and speed sums against the reports the
  traces return, bin by bin; a trace whose report() raises adds nothing.
"""
import json
import os
from collections import defaultdict

import numpy as np
import pytest

from reporter_amd import Engine, synth, tracegen

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ENV_KEYS = ("REPORT_LEVELS", "TRANSITION_LEVELS", "THRESHOLD_SEC")
with open(os.path.join(GOLD, "report_cases.json")) as _f:
    REPORT_CASES = [c for c in json.load(_f) if c["match_output"] is not None]
ENVS = sorted({json.dumps(c["env"], sort_keys=True) for c in REPORT_CASES})


def _typed(c):
    """A recorded Match output the kernel takes: every field of the JSON type
    the matcher itself emits (otm_report_segments_device hands the others
    back with code 0, "not typed")."""
    last = json.loads(c["request"]).get("trace", [{}])[-1]
    if not isinstance(last.get("time"), (int, float)) or isinstance(last.get("time"), bool):
        return False  # report() reads trace[-1]['time'] (py/reporter_service.py:116)
    m = json.loads(c["match_output"])
    segs = m.get("segments") if isinstance(m, dict) else None
    return isinstance(segs, list) and all(
        isinstance(s, dict) and isinstance(s.get("length"), int) and isinstance(s.get("queue_length"), int)
        and isinstance(s.get("begin_shape_index"), int) and s.get("begin_shape_index") >= 0
        and not isinstance(s.get("start_time"), bool) and isinstance(s.get("start_time"), (int, float))
        and not isinstance(s.get("end_time"), bool) and isinstance(s.get("end_time"), (int, float))
        for s in segs)


# the recorded cases outside the kernel's types, by name: "passthrough" hands
# report() segments with fields of other JSON types that it only passes
# through; "last_point_no_time" has no last time (report() raises KeyError:
# the host path answers it)
UNTYPED = {"passthrough", "last_point_no_time"}


def _set_env(monkeypatch, env):
    for k in ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("env_key", ENVS)
def test_k_report_reproduces_reference_cases(small_graph, monkeypatch, capfd, env_key):
    env = json.loads(env_key)
    cases = [c for c in REPORT_CASES if json.dumps(c["env"], sort_keys=True) == env_key]
    _set_env(monkeypatch, env)
    skipped = []
    with Engine(graph_path=small_graph) as eng:
        capfd.readouterr()
        for c in cases:
            (code, body), = eng.report_segments_device([(c["request"], c["match_output"])])
            out, err = capfd.readouterr()
            if code == 0:
                assert body.startswith("not typed"), body
                skipped.append(c["name"])
                continue
            assert (code, body) == (c["code"], c["body"]), c["name"]
            assert err == c["stderr"], c["name"]
        # and all of them in one launch
        got = eng.report_segments_device([(c["request"], c["match_output"]) for c in cases])
        capfd.readouterr()
        for c, (code, body) in zip(cases, got):
            if code:
                assert (code, body) == (c["code"], c["body"]), c["name"]
    # every recorded case whose Match output has the matcher's own JSON types
    # ran on the kernel; the skipped ones are exactly the untyped ones, by name
    assert sorted(skipped) == sorted(c["name"] for c in cases if not _typed(c)), skipped
    assert set(skipped) <= UNTYPED


def test_k_report_typed_coverage():
    """Which recorded cases the kernel cannot take: only Match outputs with a
    field of another JSON type than the matcher emits."""
    from reporter_amd import _lib  # noqa: F401
    assert {c["name"] for c in REPORT_CASES if not _typed(c)} == UNTYPED


@pytest.mark.parametrize("env_key", ENVS)
def test_matched_traces_under_env(small_graph, oracle, results_equal, monkeypatch, env_key):
    env = json.loads(env_key)
    _set_env(monkeypatch, env)
    b = synth.make_traces(small_graph, 150, 80, interval_s=5.0, noise_sigma_m=15.0, accuracy=15.0, seed=61)
    with Engine(graph_path=small_graph) as eng:
        res = eng.match(b)
    orc = oracle.match_batch(oracle.Graph(small_graph), b, rc=oracle.report_cfg_from_env(env), nthreads=4)
    results_equal(orc, res, "env %s" % env_key)
    assert len(res.reports) > 0 or env.get("REPORT_LEVELS") == "1"


def test_config1_generate_test_trace_requests(small_graph, oracle):
    """BASELINE config 1: py/generate_test_trace.py's synthesize_gps traces
    (tracegen restates :31-73; one point per edge end, accuracy 0) through the
    /report path on the GPU, byte-equal to the oracle's handle_request."""
    bodies = tracegen.config1_requests(small_graph, n_traces=100)
    g = oracle.Graph(small_graph)
    with Engine(graph_path=small_graph) as eng:
        got = eng.report_batch(bodies)
    ok = 0
    for body, (code, resp) in zip(bodies, got):
        assert (code, resp) == oracle.handle_request(g, body), body[:60]
        ok += code == 200 and '"reports"' in resp
    assert ok > 20  # traces long enough for a complete segment before the 15 s trim


def _hist_of(res, ids, nbins, bin_kph):
    from reporter_amd import flush
    index_of = {int(v): i for i, v in enumerate(ids)}
    h = flush.histogram_from_reports(res.reports, index_of, len(ids), nbins, bin_kph)
    rep = res.reports
    ok = (rep["flags"] & 1) == 0
    speed = rep["length"] / (rep["t1"] - rep["t0"]) * 3.6
    ok &= speed >= 0
    sums = np.zeros(len(ids), np.int64)
    for rid, sp in zip(rep["id"][ok], speed[ok]):
        sums[index_of[int(rid)]] += int(sp * 1000.0 + 0.5)
    return h, sums


def test_histogram_bins_and_speed_sums(small_graph):
    import torch
    ids = synth.segment_ids(small_graph)
    nbins, bin_kph = 16, 10.0
    b = synth.make_traces(small_graph, 300, 100, seed=23)
    with Engine(graph_path=small_graph) as eng:
        nseg = eng.graph_info()["segments"]
        assert nseg == len(ids)
        h = torch.zeros(nseg * nbins, dtype=torch.int32, device="cuda:0")
        sums = torch.zeros(nseg, dtype=torch.int64, device="cuda:0")
        eng.hist_bind(h, nbins, bin_kph, speed_sum=sums)
        r = eng.match(b)
        eng.hist_bind(None, 0, 1.0)
        torch.cuda.synchronize()
    want_h, want_s = _hist_of(r, ids, nbins, bin_kph)
    assert want_h.sum() > 100
    np.testing.assert_array_equal(h.cpu().numpy().reshape(nseg, nbins), want_h)
    np.testing.assert_array_equal(sums.cpu().numpy(), want_s)


def test_histogram_skips_traces_whose_report_raises(small_graph, oracle, monkeypatch):
    """A trace whose clock stands still for 30 points makes the segments
    traversed meanwhile last zero seconds: report() raises ZeroDivisionError
    (500) and posts nothing, so the histogram holds only the other traces'
    reports (a trace's earlier reports are not counted either)."""
    import torch
    ids = synth.segment_ids(small_graph)
    env = {"REPORT_LEVELS": "0,1,2", "TRANSITION_LEVELS": "0,1,2"}  # local streets report too
    _set_env(monkeypatch, env)
    b = synth.make_traces(small_graph, 40, 100, interval_s=5.0, noise_sigma_m=5.0, accuracy=5.0, seed=71)
    b["time"] = b["time"].copy()
    off = b["trace_off"]
    for t in range(0, 40, 2):  # every other trace: points 20..79 share one timestamp
        b["time"][off[t] + 20:off[t] + 80] = b["time"][off[t] + 20]
    with Engine(graph_path=small_graph) as eng:
        nseg = eng.graph_info()["segments"]
        h = torch.zeros(nseg * 16, dtype=torch.int32, device="cuda:0")
        eng.hist_bind(h, 16, 10.0)
        r = eng.match(b)
        eng.hist_bind(None, 0, 1.0)
        torch.cuda.synchronize()
    orc = oracle.match_batch(oracle.Graph(small_graph), b, rc=oracle.report_cfg_from_env(env), nthreads=4)
    for f in r.traces.dtype.names:
        np.testing.assert_array_equal(r.traces[f], orc["traces"][f], err_msg=f)
    zd = (r.traces["code"] == 500) & (r.traces["error_kind"] == 1)
    assert zd.sum() >= 5
    want_h, _ = _hist_of(r, ids, 16, 10.0)
    np.testing.assert_array_equal(h.cpu().numpy().reshape(nseg, 16), want_h)


def test_capacity_regrow_redo_is_identical(small_graph, oracle, results_equal, monkeypatch):
    """Tiny starting capacities (OTM_TRANS_CAP / OTM_POOL_CAP) force the
    abort -> regrow -> redo path; a small batch and then a larger one on the
    same engine must equal the oracle, histogram included (the aborted
    attempts add nothing)."""
    import torch
    ids = synth.segment_ids(small_graph)
    monkeypatch.setenv("OTM_TRANS_CAP", "64")
    monkeypatch.setenv("OTM_POOL_CAP", "16")
    small = synth.make_traces(small_graph, 20, 40, seed=81)
    large = synth.make_traces(small_graph, 250, 100, seed=82)
    g = oracle.Graph(small_graph)
    with Engine(graph_path=small_graph) as eng:
        nseg = eng.graph_info()["segments"]
        h = torch.zeros(nseg * 16, dtype=torch.int32, device="cuda:0")
        eng.hist_bind(h, 16, 10.0)
        for b in (small, large):
            h.zero_()
            r = eng.match(b)
            torch.cuda.synchronize()
            results_equal(oracle.match_batch(g, b, nthreads=4), r, "regrow")
            want_h, _ = _hist_of(r, ids, 16, 10.0)
            np.testing.assert_array_equal(h.cpu().numpy().reshape(nseg, 16), want_h)
        eng.hist_bind(None, 0, 1.0)


def test_one_engine_from_many_threads(small_graph):
    """The boundary's thread-safety contract (include/otmatch.h: an engine
    handle may be used from many threads; results of one uuid in submit
    order).  The reference serves /report from a pool of cpu_count threads
    (py/reporter_service.py:37-45).  Eight host threads call otm_report and
    otm_submit/otm_poll on ONE engine with repeated uuids; every body must be
    byte-equal to the sequential answer, and each uuid's async results must
    come back in submit order."""
    import threading
    from reporter_amd import encode_request
    b = synth.make_traces(small_graph, 48, 40, seed=91)
    bodies = []
    for t in range(48):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        # 12 uuids, each with 4 different traces
        bodies.append(encode_request("veh%d" % (t % 12), b["lat"][a:e], b["lon"][a:e],
                                     b["time"][a:e].astype(np.int64), b["accuracy"][a:e].astype(np.int32)))
    with Engine(graph_path=small_graph) as eng:
        want = [eng.report(x) for x in bodies]
        got = defaultdict(list)
        errors = []
        lock = threading.Lock()

        def sync_worker(w):
            try:
                for rep in range(3):
                    for i in range(w, 48, 8):
                        r = eng.report(bodies[i])
                        with lock:
                            got[i].append(r)
            except Exception as e:  # pragma: no cover - reported below
                errors.append(e)

        def async_worker(w):
            try:
                for i in range(w, 48, 4):
                    eng.submit(bodies[i], 1000 + i)
            except Exception as e:  # pragma: no cover
                errors.append(e)

        th = [threading.Thread(target=sync_worker, args=(w,)) for w in range(8)]
        th += [threading.Thread(target=async_worker, args=(w,)) for w in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors
        polled = []
        while len(polled) < 48:
            polled += eng.poll(64, 2000000)
    for i in range(48):
        assert got[i] == [want[i]] * 3, i
    assert sorted(tag for tag, _, _ in polled) == list(range(1000, 1048))
    for tag, code, resp in polled:
        assert (code, resp) == want[tag - 1000]
    # per uuid, results in submit order: a submitter thread w submits tags
    # w, w+4, ... in order, and a uuid's tags are i = u (mod 12) -- one thread
    # each, so the poll order of each uuid's tags is increasing
    pos = {tag: k for k, (tag, _, _) in enumerate(polled)}
    for u in range(12):
        tags = [1000 + i for i in range(u, 48, 12)]
        assert [pos[t] for t in tags] == sorted(pos[t] for t in tags), u


@pytest.mark.parametrize("workers,batch,pinned_min,gpu_min", [
    ("1", "8192", None, None), ("2", "37", None, None), ("3", "11", None, None),
    # page-locked submission slabs (every submission; or the first only, by
    # size), batches cut inside and across slabs, the GPU reader on them
    ("1", "8192", "1", None), ("2", "37", "1", None), ("3", "50", "1", "1"), ("2", "200", "full", None),
    # submissions beyond OTM_SLAB_MAX: an allocation per body, batches cut inside a submission
    ("3", "64", "slab_max", None)])
def test_async_pipeline_order_and_bodies(small_graph, monkeypatch, workers, batch, pinned_min, gpu_min):
    """otm_submit_batch / otm_poll through the async pipeline (workers on
    their own batch contexts, OTM_ASYNC_WORKERS; small OTM_ASYNC_BATCH forces
    many batches in flight): every body byte-equal to the sequential answer,
    each uuid's results in submit order, every tag once.  With
    OTM_SLAB_PINNED_MIN the submissions' slabs are page-locked and the
    worker's batches go to HBM straight from them (runs of adjacent bodies),
    mixed with staged pieces where a batch spans a small slab."""
    from reporter_amd import encode_request
    monkeypatch.setenv("OTM_ASYNC_WORKERS", workers)
    monkeypatch.setenv("OTM_ASYNC_BATCH", batch)
    if gpu_min is not None:
        monkeypatch.setenv("OTM_GPU_JSON_MIN", gpu_min)
    b = synth.make_traces(small_graph, 120, 30, seed=93)
    bodies = []
    for t in range(120):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        bodies.append(encode_request("veh%d" % (t % 17), b["lat"][a:e], b["lon"][a:e],
                                     b["time"][a:e].astype(np.int64), b["accuracy"][a:e].astype(np.int32)))
    bodies += [b"", b'{"uuid":"x","trace":[]}']
    if pinned_min == "full":  # a whole submission's slab page-locked, half of one not
        pinned_min = str(sum(len(x) for x in bodies))
    if pinned_min == "slab_max":
        monkeypatch.setenv("OTM_SLAB_MAX", "1000")
        pinned_min = "1"
    if pinned_min is not None:
        monkeypatch.setenv("OTM_SLAB_PINNED_MIN", pinned_min)
    with Engine(graph_path=small_graph) as eng:
        want = eng.report_batch(bodies)
        tags = list(range(5000, 5000 + 3 * len(bodies)))
        for r in range(3):
            if r == 1 and os.environ.get("OTM_SLAB_PINNED_MIN", "1") not in ("0", "1"):
                # the middle submission split so its slabs fall below the bound
                h = len(bodies) // 2
                eng.submit_batch(bodies[:h], tags[r * len(bodies):r * len(bodies) + h])
                eng.submit_batch(bodies[h:], tags[r * len(bodies) + h:(r + 1) * len(bodies)])
                continue
            eng.submit_batch(bodies, tags[r * len(bodies):(r + 1) * len(bodies)])
        polled = []
        while len(polled) < len(tags):
            polled += eng.poll(4096, 2000000)
    assert sorted(t for t, _, _ in polled) == tags
    for tag, code, resp in polled:
        assert (code, resp) == want[(tag - 5000) % len(bodies)]
    # results are published in submit order: tags come back increasing
    assert [t for t, _, _ in polled] == tags


def test_valhalla_module_shim(small_graph, oracle, tmp_path):
    """reporter_amd.valhalla stands in for the binding reporter_service.py
    imports: Configure (:279), SegmentMatcher() (:52), Match (:112) returns
    the oracle's Match JSON; a matcher error raises (report() -> 500)."""
    from reporter_amd import encode_request, valhalla, write_config
    b = synth.make_traces(small_graph, 6, 40, seed=97)
    g = oracle.Graph(small_graph)
    valhalla.Configure(write_config(str(tmp_path / "cfg.json"), small_graph))
    m = valhalla.SegmentMatcher()
    for t in range(6):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        body = encode_request("v%d" % t, b["lat"][a:e], b["lon"][a:e], b["time"][a:e].astype(np.int64),
                              b["accuracy"][a:e].astype(np.int32))
        code, want = oracle.match_json(g, body)
        assert code == 200 and m.Match(body.decode()) == want
    with pytest.raises(RuntimeError):
        m.Match('{"uuid":"x","trace":[{"lat":1}]}')


def _gpu_count():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_gpu_count() < 2, reason="needs a second GPU (the gpurun box has one; the driver's node has 8)")
def test_engine_on_device_1_json_and_async(small_graph):
    """An engine on device 1: otm_report_batch and the async
    workers (new host threads, which start on device 0) create their buffers,
    page-locked staging and copy streams on the engine's device; answers
    byte-equal to a device-0 engine's."""
    from reporter_amd import encode_request
    b = synth.make_traces(small_graph, 80, 30, seed=97)
    bodies = []
    for t in range(80):
        a, e = b["trace_off"][t], b["trace_off"][t + 1]
        bodies.append(encode_request("veh%d" % t, b["lat"][a:e], b["lon"][a:e], b["time"][a:e].astype(np.int64),
                                     b["accuracy"][a:e].astype(np.int32)))
    with Engine(graph_path=small_graph, device=0) as e0:
        want = e0.report_batch(bodies)
    with Engine(graph_path=small_graph, device=1) as e1:
        assert e1.report_batch(bodies) == want
        tags = list(range(len(bodies)))
        e1.submit_batch(bodies, tags)
        polled = []
        while len(polled) < len(tags):
            polled += e1.poll(4096, 2000000)
        assert sorted((t, c, s) for t, c, s in polled) == [(t, want[t][0], want[t][1]) for t in tags]


@pytest.mark.parametrize("size", ["small", "pieces"])
def test_request_arena_report_and_submit(small_graph, oracle, monkeypatch, size):
    """Bodies written into a library-owned request arena
    (otm_request_arena_alloc) go to HBM straight from it, through
    otm_report_batch (direct pieces, cut at 16 MB: "pieces" spans more than
    one) and otm_submit_batch (referenced, not copied): every response
    byte-equal to the copied path's and to the oracle's, a malformed body and
    a body for the host readers among them, and the arena reusable after."""
    from reporter_amd import RequestArena, encode_request
    n, pts = (60, 40) if size == "small" else (2600, 100)  # "pieces": ~17 MB of bodies
    b = synth.make_traces(small_graph, n, pts, seed=97)
    off = b["trace_off"]
    bodies = [encode_request("veh%d" % t, b["lat"][off[t]:off[t + 1]], b["lon"][off[t]:off[t + 1]],
                             b["time"][off[t]:off[t + 1]].astype(np.int64),
                             b["accuracy"][off[t]:off[t + 1]].astype(np.int32)) for t in range(n)]
    bodies[3] = b"{"
    bodies[7] = bodies[7].replace(b'"trace":', b'"trace" :')
    if size == "pieces":
        assert sum(len(x) for x in bodies) > (16 << 20)
    with Engine(graph_path=small_graph) as eng:
        want = eng.report_batch(bodies)
        with RequestArena(bodies) as ar:
            assert eng.report_batch(ar) == want
            assert eng.report_batch(ar) == want  # (reused)
            tags = list(range(100, 100 + n))
            eng.submit_batch(ar, tags)
            polled = []
            while len(polled) < n:
                polled += eng.poll(4096, 2000000)
        assert [t for t, _, _ in polled] == tags
        assert [(c, r) for _, c, r in polled] == want
        # a submission keeps its arena alive past the caller's release
        ar2 = RequestArena(bodies[:50])
        eng.submit_batch(ar2, list(range(50)))
        ar2.release()
        polled = []
        while len(polled) < 50:
            polled += eng.poll(4096, 2000000)
        assert [(c, r) for _, c, r in polled] == want[:50]
    if size == "small":
        g = oracle.Graph(small_graph)
        for body, got in zip(bodies, want):
            assert got == oracle.handle_request(g, body), body[:60]


def test_report_batch_split_over_contexts(small_graph, capfd):
    """otm_report_batch over >= 2 x 2048 bodies is cut into one chunk per
    batch context (report_many_split: the chunks run concurrently, their copies
    to HBM in chunk order on one copy stream): every response byte-equal to the
    same call run as one batch (an engine counting its kernels is not split),
    from bytes objects and from a request arena, the same stderr lines, with a
    malformed body and a host-reader body among them; and the engine's async
    pipeline still runs on the same contexts after."""
    from reporter_amd import RequestArena, _lib, encode_request
    L = _lib.lib()
    n, pts = 6200, 30
    b = synth.make_traces(small_graph, n, pts, seed=41)
    off = b["trace_off"]
    bodies = [encode_request("veh%d" % t, b["lat"][off[t]:off[t + 1]], b["lon"][off[t]:off[t + 1]],
                             b["time"][off[t]:off[t + 1]].astype(np.int64),
                             b["accuracy"][off[t]:off[t + 1]].astype(np.int32)) for t in range(n)]
    bodies[5] = b"{"
    bodies[4000] = bodies[4000].replace(b'"trace":', b'"trace" :')
    with Engine(graph_path=small_graph) as eng:
        capfd.readouterr()
        got = eng.report_batch(bodies)
        split_err = capfd.readouterr().err
        assert L.otm_debug_last_split(eng.h) >= 2
        with RequestArena(bodies) as ar:
            assert eng.report_batch(ar) == got
        assert L.otm_debug_last_split(eng.h) >= 2
        eng.set_counting(True)
        capfd.readouterr()
        want = eng.report_batch(bodies)
        one_err = capfd.readouterr().err
        assert L.otm_debug_last_split(eng.h) == 1
        eng.set_counting(False)
        eng.submit_batch(bodies[:3000], list(range(3000)))
        polled = []
        while len(polled) < 3000:
            polled += eng.poll(4096, 2000000)
        assert [(c, r) for _, c, r in polled] == want[:3000]
        assert eng.report_batch(bodies) == want  # (split again, beside the running workers)
    assert got == want
    assert sorted(split_err.splitlines()) == sorted(one_err.splitlines())
