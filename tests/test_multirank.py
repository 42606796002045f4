"""world_size-2 gloo rehearsal of the multi-GPU path on CPU.

Each rank takes its uuid shard (murmur2 partitioner), matches it (here with
the CPU oracle: there is no GPU in this container), bins its datastore
reports per segment and joins the histogram reduction of
reporter_amd.flush.  The reduced shards must equal the histogram of the whole
fleet computed by one process, and the uuid shards must partition the fleet.
"""
import os
import struct

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NV, NPTS, NBINS, BIN_KPH = 120, 60, 16, 10.0


def seg_ids(graph):
    raw = np.fromfile(graph, dtype=np.uint8)
    fmt = "<8sII4i2iq3d4dQ"
    hs = struct.calcsize(fmt)
    o, n = struct.unpack_from("<QQ", raw, hs + 16 * 17)  # OTMG_SEG_ID
    return np.frombuffer(raw, dtype=np.uint64, count=n // 8, offset=o)


def _fleet_hist(graph, vehicle_ids, index_of):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import pyoracle
    from reporter_amd import flush, synth
    b = synth.make_traces(graph, len(vehicle_ids), NPTS, vehicle_ids=vehicle_ids, seed=31)
    r = pyoracle.match_batch(pyoracle.Graph(graph), b, nthreads=2)
    return flush.histogram_from_reports(r["reports"], index_of, len(seg_ids(graph)), NBINS, BIN_KPH)


def _worker(rank, world, graph, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from reporter_amd import flush, synth
    ids = seg_ids(graph)
    index_of = {int(v): i for i, v in enumerate(ids)}
    mine = synth.shard_vehicle_ids(NV // world, rank, world)
    h = _fleet_hist(graph, mine, index_of)
    rows = flush.padded_segments(len(ids), world)
    full = torch.zeros(rows * NBINS, dtype=torch.int32)
    full[:len(ids) * NBINS] = torch.from_numpy(h.reshape(-1).astype(np.int32))
    part = flush.reduce_histograms(full)
    np.save(os.path.join(out_dir, "part%d.npy" % rank), part.numpy())
    np.save(os.path.join(out_dir, "ids%d.npy" % rank), mine)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_histogram_reduction(small_graph, tmp_path):
    world = 2
    port = 29500 + os.getpid() % 1000
    mp.start_processes(_worker, args=(world, small_graph, port, str(tmp_path)), nprocs=world, start_method="spawn")
    from reporter_amd import flush
    ids0, ids1 = np.load(tmp_path / "ids0.npy"), np.load(tmp_path / "ids1.npy")
    assert not set(ids0.tolist()) & set(ids1.tolist())
    allv = np.concatenate([ids0, ids1])
    sids = seg_ids(small_graph)
    index_of = {int(v): i for i, v in enumerate(sids)}
    ref = _fleet_hist(small_graph, allv, index_of).reshape(-1)
    rows = flush.padded_segments(len(sids), world)
    ref_p = np.zeros(rows * NBINS, np.int64)
    ref_p[:ref.size] = ref
    got = np.concatenate([np.load(tmp_path / "part0.npy"), np.load(tmp_path / "part1.npy")])
    assert got.sum() > 0
    assert np.array_equal(got, ref_p)
