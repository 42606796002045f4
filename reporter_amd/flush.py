"""Cross-GPU flush of per-segment speed histograms.

Traces are sharded by uuid (Kafka's murmur2 key partitioner, the same split
the reference's keyed `formatted` topic gives its batchers,
Reporter.java:97,102); each GPU matches its shard with no data-path exchange.
The one collective is this reduction of the per-segment histograms before the
datastore flush: a reduce-scatter, so that rank r ends up owning segments
[r*S/W, (r+1)*S/W) and flushes only those.  The reference never aggregates
(its datastore POST is a TODO, docker-compose.yml:17); the records a rank
flushes are written by reporter_amd.datastore.

Buffers (S = segments padded to a multiple of the world size W, B bins):
  counts     int32 [S * B]  -> each rank's slice int32 [S * B / W]
  speed sums int64 [S]      -> int64 [S / W]   (1/1000 km/h, fixed point)
One dist.reduce_scatter_tensor per buffer: RCCL over xGMI with backend
"nccl", the same collective in gloo (CPU tests).  At config 2 (13.6k
segments, 16 bins) that is 0.87 MB + 0.11 MB per flush; at a 1M-segment
metro graph 64 MB + 8 MB, one ring pass per flush window.
"""
import time

import torch
import torch.distributed as dist


def padded_segments(n_segments, world):
    """Histogram rows padded to a multiple of the world size."""
    return (n_segments + world - 1) // world * world


def reduce_histograms(hist, out=None, speed_sum=None, speed_out=None):
    """Sum `hist` ([S_pad * nbins], int32) -- and `speed_sum` ([S_pad], int64)
    when given -- over all ranks; return this rank's slice of the sums
    ([S_pad * nbins / W], and [S_pad / W]): rows [r*S_pad/W, (r+1)*S_pad/W)."""
    world = dist.get_world_size()
    n = hist.numel() // world
    if hist.numel() % world:
        raise ValueError("histogram rows must be padded to a multiple of the world size")
    if out is None:
        out = torch.empty(n, dtype=hist.dtype, device=hist.device)
    dist.reduce_scatter_tensor(out, hist)
    if speed_sum is None:
        return out
    if speed_out is None:
        speed_out = torch.empty(speed_sum.numel() // world, dtype=speed_sum.dtype, device=speed_sum.device)
    dist.reduce_scatter_tensor(speed_out, speed_sum)
    return out, speed_out


def close_window(t_start, hist, hist_out=None, speed_sum=None, speed_out=None, sync=None):
    """End of a timed window of the multi-GPU bench (bench.py): wait for this
    rank's work (`sync`, e.g. torch.cuda.synchronize), then -- over more than
    one rank -- the window's histogram flush (reduce_histograms: RCCL over
    xGMI, or gloo) and a barrier.  Returns the window's seconds since
    `t_start` (time.perf_counter) as the MAX over ranks: every rank gets the
    same figure, the slowest rank's."""
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if sync:
        sync()
    if multi:
        reduce_histograms(hist, out=hist_out, speed_sum=speed_sum, speed_out=speed_out)
        if sync:
            sync()
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if multi:
        t = torch.tensor([elapsed], dtype=torch.float64, device=hist.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def histogram_from_reports(reports, seg_index_of_id, n_rows, nbins, bin_kph):
    """Host restatement of k_report's binning (the GPU builds the histogram
    in the same pass as report()): one count per datastore report with a
    valid t1 and speed >= 0, bin = floor(kph / bin_kph) clamped to nbins-1."""
    return histograms_from_reports(reports, seg_index_of_id, n_rows, nbins, bin_kph)[0]


def histograms_from_reports(reports, seg_index_of_id, n_rows, nbins, bin_kph):
    """(counts int64 [n_rows, nbins], speed sums int64 [n_rows] in 1/1000
    km/h) of the reports, binned as k_report bins them."""
    import numpy as np
    h = np.zeros((n_rows, nbins), np.int64)
    sums = np.zeros(n_rows, np.int64)
    ok = (reports["flags"] & 1) == 0
    speed = reports["length"] / (reports["t1"] - reports["t0"]) * 3.6
    ok &= speed >= 0
    for rid, sp in zip(reports["id"][ok], speed[ok]):
        b = min(max(int(sp / bin_kph), 0), nbins - 1)
        row = seg_index_of_id[int(rid)]
        h[row, b] += 1
        sums[row] += int(sp * 1000.0 + 0.5)
    return h, sums
