"""How much SURVEY Appendix B's node snap would change (departures).

Runs the CPU oracle over a slice of a config's batch and counts candidates whose
projection is clamped to an edge end (offset 0 or the edge length) -- the ones
meili would snap to the node and share among the node's incident edges -- and
matched states at an edge end.  CPU only (oracle = test infrastructure).

    python scripts/node_snap_stats.py [config] [vehicles]
"""
import os
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import pyoracle  # noqa: E402
from reporter_amd import synth  # noqa: E402


def section(path, idx, dtype):
    raw = np.fromfile(path, dtype=np.uint8)
    hs = struct.calcsize("<8sII4i2iq3d4dQ")
    o, n = struct.unpack_from("<QQ", raw, hs + 16 * idx)
    return np.frombuffer(raw, dtype=dtype, count=n // np.dtype(dtype).itemsize, offset=o).copy()


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    nveh = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    gpath = synth.cached_graph(cfg)
    c = synth.CONFIGS[cfg]
    t = dict(c["traces"])
    t["n_vehicles"] = min(nveh, t["n_vehicles"])
    b = synth.make_traces(gpath, **t)
    elen = section(gpath, 5, np.float32)      # OTMG_EDGE_LEN
    eto = section(gpath, 4, np.int32)         # OTMG_EDGE_TO
    efrom = section(gpath, 3, np.int32)       # OTMG_EDGE_FROM
    g = pyoracle.Graph(gpath)
    p = pyoracle.params(**c.get("meili", {}))
    r = pyoracle.match_batch(g, b, p=p, keep_stages=True)
    K = pyoracle.KMAX
    nc = r["ncand"]
    P = len(nc)
    mask = np.arange(K)[None, :] < nc[:, None]
    e = r["cand_edge"].reshape(P, K)
    o = r["cand_off"].reshape(P, K)
    ee = np.where(mask, e, 0)
    at_start = mask & (o == 0.0)
    at_end = mask & (o == elen[ee])
    ends = at_start | at_end
    # node each end-candidate sits on; candidates of one point on the same node collapse into one
    node = np.where(at_start, efrom[ee], np.where(at_end, eto[ee], -1))
    merged = 0
    for i in np.nonzero(ends.any(1))[0]:
        nn = node[i][ends[i]]
        merged += len(nn) - len(np.unique(nn))
    st = r["state"]
    m = st >= 0
    idx = np.nonzero(m)[0]
    se = e[idx, st[idx]]
    so = o[idx, st[idx]]
    st_end = (so == 0.0) | (so == elen[se])
    print("config %d, %d vehicles, %d points, %d candidates" % (cfg, t["n_vehicles"], P, int(mask.sum())))
    print("candidates at an edge end: %.1f %%" % (100.0 * ends.sum() / max(1, mask.sum())))
    print("candidates a node snap would merge away: %.1f %%" % (100.0 * merged / max(1, mask.sum())))
    print("matched states at an edge end: %.1f %%" % (100.0 * st_end.sum() / max(1, len(idx))))


if __name__ == "__main__":
    main()
