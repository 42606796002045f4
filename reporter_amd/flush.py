"""Cross-GPU flush of per-segment speed histograms.

Traces are sharded by uuid (Kafka's murmur2 key partitioner, the same split
the reference's keyed `formatted` topic gives its batchers,
Reporter.java:97,102); each GPU matches its shard with no data-path exchange.
The one collective is this reduction of the per-segment histograms before the
datastore flush: a reduce-scatter, so that rank r ends up owning segments
[r*S/W, (r+1)*S/W) and flushes only those.  The reference never aggregates
(its datastore POST is a TODO, docker-compose.yml:17).
"""
import torch
import torch.distributed as dist


def padded_segments(n_segments, world):
    """Histogram rows padded to a multiple of the world size."""
    return (n_segments + world - 1) // world * world


def reduce_histograms(hist, out=None):
    """Sum `hist` ([S_pad * nbins], int32) over all ranks; return this rank's
    slice of the sum ([S_pad * nbins / W]).  RCCL (backend "nccl") does it
    with one reduce-scatter over xGMI; gloo (CPU tests) with all-reduce +
    slice, which yields the same slice."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    n = hist.numel() // world
    if out is None:
        out = torch.empty(n, dtype=hist.dtype, device=hist.device)
    if dist.get_backend() == "nccl":
        dist.reduce_scatter_tensor(out, hist)
    else:
        tmp = hist.clone()
        dist.all_reduce(tmp)
        out.copy_(tmp[rank * n:(rank + 1) * n])
    return out


def histogram_from_reports(reports, seg_index_of_id, n_rows, nbins, bin_kph):
    """Host restatement of k_report's binning (the GPU builds the histogram
    in the same pass as report()): one count per datastore report with a
    valid t1 and speed >= 0, bin = floor(kph / bin_kph) clamped to nbins-1."""
    import numpy as np
    h = np.zeros((n_rows, nbins), np.int64)
    ok = (reports["flags"] & 1) == 0
    speed = reports["length"] / (reports["t1"] - reports["t0"]) * 3.6
    ok &= speed >= 0
    for rid, sp in zip(reports["id"][ok], speed[ok]):
        b = min(max(int(sp / bin_kph), 0), nbins - 1)
        h[seg_index_of_id[int(rid)], b] += 1
    return h
