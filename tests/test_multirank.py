"""world_size-2 gloo rehearsal of the multi-GPU path on CPU.

Each rank takes its uuid shard (murmur2 partitioner), matches it (here with
the CPU oracle: there is no GPU in this container), bins its datastore
reports per segment (counts and speed sums) and joins the reduction of
reporter_amd.flush: the same dist.reduce_scatter_tensor that RCCL runs on the
GPUs, here over gloo.  Rank r must end up with rows [r*S/W, (r+1)*S/W) of the
whole fleet's histogram computed by one process, the uuid shards must
partition the fleet, and each rank's datastore flush body must describe
exactly its rows.
"""
import json
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NV, NPTS, NBINS, BIN_KPH = 120, 60, 16, 10.0


def _fleet_hist(graph, vehicle_ids, index_of, n_rows):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import pyoracle
    from reporter_amd import flush, synth
    b = synth.make_traces(graph, len(vehicle_ids), NPTS, vehicle_ids=vehicle_ids, seed=31)
    r = pyoracle.match_batch(pyoracle.Graph(graph), b, nthreads=2)
    return flush.histograms_from_reports(r["reports"], index_of, n_rows, NBINS, BIN_KPH)


def _worker(rank, world, graph, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from reporter_amd import datastore, flush, synth
    ids = synth.segment_ids(graph)
    index_of = {int(v): i for i, v in enumerate(ids)}
    mine = synth.shard_vehicle_ids(NV // world, rank, world)
    rows = flush.padded_segments(len(ids), world)
    h, s = _fleet_hist(graph, mine, index_of, rows)
    counts = torch.from_numpy(h.reshape(-1).astype(np.int32))
    sums = torch.from_numpy(s)
    part, spart = flush.reduce_histograms(counts, speed_sum=sums)
    assert part.numel() == rows * NBINS // world and spart.numel() == rows // world
    np.save(os.path.join(out_dir, "part%d.npy" % rank), part.numpy())
    np.save(os.path.join(out_dir, "sums%d.npy" % rank), spart.numpy())
    np.save(os.path.join(out_dir, "ids%d.npy" % rank), mine)
    body = datastore.serialize(datastore.flush_records(part.numpy(), spart.numpy(), ids, rank, world, NBINS,
                                                       BIN_KPH))
    with open(os.path.join(out_dir, "flush%d.json" % rank), "wb") as f:
        f.write(body)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_histogram_reduction(small_graph, tmp_path):
    world = 2
    port = 29500 + os.getpid() % 1000
    mp.start_processes(_worker, args=(world, small_graph, port, str(tmp_path)), nprocs=world, start_method="spawn")
    from reporter_amd import flush, synth
    ids0, ids1 = np.load(tmp_path / "ids0.npy"), np.load(tmp_path / "ids1.npy")
    assert not set(ids0.tolist()) & set(ids1.tolist())
    allv = np.concatenate([ids0, ids1])
    sids = synth.segment_ids(small_graph)
    index_of = {int(v): i for i, v in enumerate(sids)}
    rows = flush.padded_segments(len(sids), world)
    ref_h, ref_s = _fleet_hist(small_graph, allv, index_of, rows)
    got = np.concatenate([np.load(tmp_path / "part0.npy"), np.load(tmp_path / "part1.npy")])
    got_s = np.concatenate([np.load(tmp_path / "sums0.npy"), np.load(tmp_path / "sums1.npy")])
    assert got.sum() > 0
    assert np.array_equal(got, ref_h.reshape(-1))
    assert np.array_equal(got_s, ref_s)
    # the flush bodies: each rank names only its own rows, together all of them
    seen = {}
    for r in range(world):
        body = json.loads((tmp_path / ("flush%d.json" % r)).read_bytes())
        lo, hi = r * rows // world, (r + 1) * rows // world
        for rec in body["segments"]:
            row = index_of[rec["id"]]
            assert lo <= row < hi
            assert rec["bins"] == ref_h[row].tolist() and rec["count"] == int(ref_h[row].sum())
            assert rec["speed_sum_kph"] == ref_s[row] / 1000.0
            seen[row] = True
    assert len(seen) == int((ref_h.sum(axis=1) > 0).sum())


def test_datastore_post_keeps_the_secret_key(tmp_path):
    """The flush POSTs to DATASTORE_URL as configured, secret_key query
    parameter included (README.md:196-198); a local HTTP server receives it."""
    import threading
    from http.server import BaseHTTPRequestHandler, HTTPServer

    from reporter_amd import datastore
    got = {}

    class H(BaseHTTPRequestHandler):
        def do_POST(self):  # noqa: N802
            n = int(self.headers["Content-Length"])
            got["path"] = self.path
            got["type"] = self.headers["Content-type"]
            got["body"] = self.rfile.read(n)
            self.send_response(200)
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = HTTPServer(("127.0.0.1", 0), H)
    th = threading.Thread(target=srv.handle_request)
    th.start()
    body = datastore.serialize({"mode": "auto", "segments": [{"id": 8, "count": 1, "bins": [1]}]})
    status = datastore.post(body, url="http://127.0.0.1:%d/store?secret_key=abc" % srv.server_port)
    th.join()
    srv.server_close()
    assert status == 200
    assert got["path"] == "/store?secret_key=abc"
    assert got["body"] == body and got["type"].startswith("application/json")
    assert datastore.post(body, url="") is None or os.environ.get("DATASTORE_URL")


def _window_worker(rank, world, port, out_dir):
    import sys
    import time
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from reporter_amd import flush
    rows, nb = flush.padded_segments(37, world), 4
    hist = torch.arange(rows * nb, dtype=torch.int32) * (rank + 1)
    sums = torch.arange(rows, dtype=torch.int64) * 1000 * (rank + 1)
    out = torch.empty(rows * nb // world, dtype=torch.int32)
    sout = torch.empty(rows // world, dtype=torch.int64)
    dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.05 + 0.25 * rank)  # rank 1 is the slow one
    el = flush.close_window(t0, hist, hist_out=out, speed_sum=sums, speed_out=sout)
    np.save(os.path.join(out_dir, "w%d.npy" % rank), np.array([el]))
    np.save(os.path.join(out_dir, "h%d.npy" % rank), out.numpy())
    np.save(os.path.join(out_dir, "s%d.npy" % rank), sout.numpy())
    dist.destroy_process_group()


def test_bench_window_helper_max_over_ranks_and_flush(tmp_path):
    """bench.py's N > 1 timed window (flush.close_window): the histogram
    reduce-scatter runs inside it and every rank reports the slowest rank's
    time."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    world = 2
    mp.start_processes(_window_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    el = [float(np.load(str(tmp_path / ("w%d.npy" % r)))[0]) for r in range(world)]
    assert el[0] == el[1] and el[0] >= 0.3
    from reporter_amd import flush
    rows, nb = flush.padded_segments(37, world), 4
    full = np.arange(rows * nb, dtype=np.int64) * 3  # (1 + 2) x
    fs = np.arange(rows, dtype=np.int64) * 1000 * 3
    for r in range(world):
        h = np.load(str(tmp_path / ("h%d.npy" % r)))
        sm = np.load(str(tmp_path / ("s%d.npy" % r)))
        np.testing.assert_array_equal(h, full[r * rows * nb // world:(r + 1) * rows * nb // world])
        np.testing.assert_array_equal(sm, fs[r * rows // world:(r + 1) * rows // world])
