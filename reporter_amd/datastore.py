"""Datastore flush of a rank's reduced speed histograms.

The reference never posts to the datastore: DATASTORE_URL is a TODO
(docker-compose.yml:17, README.md:30,56,94), and the reports it would send
are only returned in each /report response (py/reporter_service.py:160-166,
"datastore" in README.md:135-141).  Authentication is a `secret_key` query
parameter already in the URL (README.md:196-198), so the flush posts to the
URL exactly as configured.

After flush.reduce_histograms, rank r owns segment rows
[r*S_pad/W, (r+1)*S_pad/W).  This module turns that slice into one JSON body
(segments with at least one report: id, count, speed sum and per-bin counts)
and POSTs it.  The body format is this build's own (the datastore's API is
not in the reference); it carries everything the reduced buffers hold.
"""
import json
import os
import urllib.request

import numpy as np


def rank_rows(n_segments_padded, rank, world):
    """The histogram rows rank `rank` owns after the reduce-scatter."""
    per = n_segments_padded // world
    return rank * per, (rank + 1) * per


def flush_records(counts, speed_sums, segment_ids, rank, world, nbins, bin_kph):
    """Records of one rank's slice: counts int [rows * nbins] and speed sums
    int [rows] (1/1000 km/h) as reduce_histograms returned them; segment_ids
    u64 [n_segments] of the graph (synth.segment_ids)."""
    counts = np.asarray(counts, np.int64).reshape(-1, nbins)
    sums = np.asarray(speed_sums, np.int64).reshape(-1)
    r0, _ = rank_rows(counts.shape[0] * world, rank, world)
    out = []
    tot = counts.sum(axis=1)
    for k in np.nonzero(tot > 0)[0]:
        row = r0 + int(k)
        if row >= len(segment_ids):  # padding rows never count
            continue
        out.append({"id": int(segment_ids[row]), "count": int(tot[k]),
                    "speed_sum_kph": int(sums[k]) / 1000.0,
                    "bins": [int(x) for x in counts[k]]})
    return {"mode": "auto", "bin_kph": float(bin_kph), "rank": rank, "world": world, "segments": out}


def serialize(records):
    """Compact JSON, as reporter_service.py writes its bodies (:215)."""
    return json.dumps(records, separators=(",", ":")).encode("utf-8")


def post(body, url=None, timeout=10.0):
    """POST a flush body to the datastore (url or env DATASTORE_URL, its
    secret_key query parameter included).  Returns the HTTP status; raises on
    transport errors.  No URL configured: nothing is sent (returns None), as
    in the reference."""
    url = url or os.environ.get("DATASTORE_URL")
    if not url:
        return None
    req = urllib.request.Request(url, data=body, method="POST",
                                 headers={"Content-type": "application/json;charset=utf-8"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.status
