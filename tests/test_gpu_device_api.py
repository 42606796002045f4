"""otm_match_device (the device-resident entry bench.py's `value` times):
inputs already in HBM as torch tensors, launched on the engine's own stream,
on a caller's torch stream, or on a library stream with a hardware queue of
its own (otm_stream_create), and fetched with otm_fetch_results -- every
result field equal to the host-batch path's (otm_match_soa) on the same
batch, which the parity tests hold to the oracle."""
import numpy as np
import pytest

from reporter_amd import Engine, _lib, synth

pytestmark = pytest.mark.gpu


def _fields_equal(a, b):
    assert a.shape == b.shape
    for name in a.dtype.names:
        assert np.array_equal(a[name], b[name]), name


@pytest.mark.parametrize("stream_kind", ["engine", "torch", "own_queue"])
def test_match_device_equals_host_batch(small_graph, stream_kind):
    import torch
    b = synth.make_traces(small_graph, 400, 60, seed=11)
    dt = {"trace_off": np.int64, "lat": np.float32, "lon": np.float32, "time": np.float64, "accuracy": np.float32}
    arr = {k: np.ascontiguousarray(b[k], dtype=v) for k, v in dt.items()}
    dev = torch.device("cuda:0")
    L = _lib.lib()
    with Engine(graph_path=small_graph) as eng:
        r = eng.match(arr)
        want = (r.traces.copy(), r.segments.copy(), r.reports.copy(), r.way_ids.copy())
        t = {k: torch.from_numpy(v).to(dev) for k, v in arr.items()}
        torch.cuda.synchronize(dev)
        own = None
        if stream_kind == "engine":
            s = None
        elif stream_kind == "torch":
            ts = torch.cuda.Stream(dev)
            s = ts.cuda_stream
        else:
            own = L.otm_stream_create(eng.h, 1)
            assert own
            s = own
        for _ in range(2):  # (a second batch on the same context and stream)
            eng.match_device(t["trace_off"], t["lat"], t["lon"], t["time"], t["accuracy"], stream=s)
            torch.cuda.synchronize(dev)
            g = eng.fetch()
            _fields_equal(g.traces, want[0])
            _fields_equal(g.segments, want[1])
            _fields_equal(g.reports, want[2])
            assert np.array_equal(g.way_ids, want[3])
        if own:
            L.otm_stream_destroy(own)
    assert len(want[1]) > 0 and len(want[2]) > 0
