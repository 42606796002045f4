"""A hand-built .otmg writer for tests (include/otm_graph_format.h, version 2).

The synthetic generator (reporter_amd/csrc/synth_graph.cpp) makes city-sized
graphs; the golden cases that pin a rule by hand need a graph small enough to
reason about: a few nodes, straight edges, chosen OSMLR segments.  This module
lays such a graph out in the file format every reader uses (engine and
oracle), with the same grid construction and heading convention as the
generator.
"""
import math
import struct

import numpy as np

MAGIC = b"OTMGRAPH"
VERSION = 2
EDGE_INTERNAL, SEG_BEGIN, SEG_END = 0x01, 0x02, 0x04
_HDR = "<8sII6iq3d4dQ"
N_SECTIONS = 25
MPD = 20037581.187 / 180.0


def _bearing(la0, lo0, la1, lo1):
    dy = la1 - la0
    dx = (lo1 - lo0) * math.cos(math.radians(la0))
    b = math.degrees(math.atan2(dx, dy))
    return int(round(b)) % 360


def write(path, nodes, edges, segments, cell_deg=0.0005):
    """nodes: [(lat, lon)]; edges: dicts with from, to, optional shape
    [(lat, lon), ...] (default: the straight line between the nodes), way,
    seg (index into segments or -1), seg_pos, flags, level; segments: [(id,
    length_m)].  Edges are re-sorted by from node (CSR order); returns the
    list mapping each given edge to its id in the file."""
    NN = len(nodes)
    order = sorted(range(len(edges)), key=lambda i: (edges[i]["from"], i))
    rank = {i: r for r, i in enumerate(order)}
    nlat = np.array([n[0] for n in nodes], np.float32)
    nlon = np.array([n[1] for n in nodes], np.float32)
    out_off = np.zeros(NN + 1, np.int32)
    efrom, eto, elen, eshape, eway, eseg, epos, efl, elev, espd, eopp = ([] for _ in range(11))
    slat, slon, scum, hout, hin = [], [], [], [], []
    for i in order:
        e = edges[i]
        sh = e.get("shape") or [nodes[e["from"]], nodes[e["to"]]]
        sh = [(np.float32(a), np.float32(b)) for a, b in sh]
        eshape.append(len(slat))
        cum = 0.0
        for k, (la, lo) in enumerate(sh):
            if k:
                pla, plo = sh[k - 1]
                dy = (float(la) - float(pla)) * MPD
                dx = (float(lo) - float(plo)) * MPD * math.cos(math.radians(0.5 * (float(la) + float(pla))))
                cum += math.hypot(dx, dy)
            slat.append(la)
            slon.append(lo)
            scum.append(np.float32(cum))
        efrom.append(e["from"])
        eto.append(e["to"])
        elen.append(scum[-1])
        eway.append(e.get("way", 1000 + i))
        eseg.append(e.get("seg", -1))
        epos.append(e.get("seg_pos", 0))
        efl.append(e.get("flags", 0))
        elev.append(e.get("level", 2))
        espd.append(40.0)
        eopp.append(-1)
        hout.append(_bearing(float(sh[0][0]), float(sh[0][1]), float(sh[1][0]), float(sh[1][1])))
        hin.append(_bearing(float(sh[-2][0]), float(sh[-2][1]), float(sh[-1][0]), float(sh[-1][1])))
        out_off[e["from"] + 1] += 1
    eshape.append(len(slat))
    out_off = np.cumsum(out_off).astype(np.int32)
    NE = len(order)
    slat = np.array(slat, np.float32)
    slon = np.array(slon, np.float32)
    # grid: as synth_graph.cpp (cells a shape segment's lat/lon box overlaps)
    lat0 = math.floor(float(slat.min()) / cell_deg) * cell_deg - cell_deg
    lon0 = math.floor(float(slon.min()) / cell_deg) * cell_deg - cell_deg
    rows = int(math.ceil((float(slat.max()) - lat0) / cell_deg)) + 2
    cols = int(math.ceil((float(slon.max()) - lon0) / cell_deg)) + 2
    cells = [[] for _ in range(rows * cols)]
    for k in range(NE):
        for s in range(eshape[k + 1] - eshape[k] - 1):
            a = eshape[k] + s
            la0, la1 = sorted((float(slat[a]), float(slat[a + 1])))
            lo0, lo1 = sorted((float(slon[a]), float(slon[a + 1])))
            for r in range(int(math.floor((la0 - lat0) / cell_deg)), int(math.floor((la1 - lat0) / cell_deg)) + 1):
                for c in range(int(math.floor((lo0 - lon0) / cell_deg)), int(math.floor((lo1 - lon0) / cell_deg)) + 1):
                    cells[r * cols + c].append((k << 4) | s)
    cell_off = np.zeros(rows * cols + 1, np.int64)
    cell_off[1:] = np.cumsum([len(c) for c in cells])
    cell_ent = np.array([x for c in cells for x in c], np.uint32)
    seg_id = np.array([s[0] for s in segments], np.uint64)
    # a segment length of None: the sum of its edges' lengths
    seg_len = np.zeros(len(segments), np.float32)
    for g, s in enumerate(segments):
        if s[1] is not None:
            seg_len[g] = s[1]
        else:
            seg_len[g] = sum(float(elen[r]) for r, i in enumerate(order) if edges[i].get("seg", -1) == g)
    gfirst = np.zeros(len(segments), np.int32)
    gn = np.zeros(len(segments), np.int32)
    for r, i in enumerate(order):
        sgi = edges[i].get("seg", -1)
        if sgi >= 0:
            if gn[sgi] == 0 or edges[i].get("seg_pos", 0) == 0:
                gfirst[sgi] = r
            gn[sgi] += 1
    secs = [nlat, nlon, out_off, np.array(efrom, np.int32), np.array(eto, np.int32), np.array(elen, np.float32),
            np.array(eshape, np.int32), np.array(eway, np.int64), np.array(eseg, np.int32), np.array(epos, np.int32),
            np.array(efl, np.uint8), np.array(elev, np.uint8), np.array(espd, np.float32),
            np.array(eopp, np.int32), slat, slon, np.array(scum, np.float32), seg_id, seg_len, gfirst, gn,
            cell_off, cell_ent, np.array(hout, np.uint16), np.array(hin, np.uint16)]
    assert len(secs) == N_SECTIONS
    hdr_bytes = struct.calcsize(_HDR) + 16 * N_SECTIONS
    align = lambda x: (x + 255) & ~255
    off = align(hdr_bytes)
    desc = []
    for a in secs:
        desc.append((off, a.nbytes))
        off = align(off + a.nbytes)
    bbox = (float(nlat.min()), float(nlon.min()), float(nlat.max()), float(nlon.max()))
    hdr = struct.pack(_HDR, MAGIC, VERSION, hdr_bytes, NN, NE, len(slat), len(segments), rows, cols,
                      len(cell_ent), lat0, lon0, cell_deg, *bbox, 0)
    hdr += b"".join(struct.pack("<QQ", o, n) for o, n in desc)
    with open(path, "wb") as f:
        f.write(hdr)
        pos = len(hdr)
        for (o, n), a in zip(desc, secs):
            f.write(b"\0" * (o - pos))
            f.write(a.tobytes())
            pos = o + n
    return [rank[i] for i in range(len(edges))]


def straight_road(path, lat=40.0, lon0=0.0, step_deg=0.001, n_nodes=5, two_way=True, seg_per_edge=True):
    """An east-west road of n_nodes - 1 straight edges; each forward edge its
    own level-0 OSMLR segment (ids (i + 1) << 3) when seg_per_edge, else one
    segment over the whole road.  Reverse edges carry no segment.  Returns
    (path, forward edge ids in the file)."""
    nodes = [(lat, lon0 + i * step_deg) for i in range(n_nodes)]
    edges, segs = [], []
    for i in range(n_nodes - 1):
        if seg_per_edge:
            sg, pos, fl = len(segs), 0, SEG_BEGIN | SEG_END
            segs.append(((i + 1) << 3, None))
        else:
            if not segs:
                segs.append((1 << 3, None))
            sg, pos = 0, i
            fl = (SEG_BEGIN if i == 0 else 0) | (SEG_END if i == n_nodes - 2 else 0)
        edges.append(dict(**{"from": i, "to": i + 1}, way=100 + i, seg=sg, seg_pos=pos, flags=fl, level=0))
        if two_way:
            edges.append(dict(**{"from": i + 1, "to": i}, way=100 + i, seg=-1, level=0))
    ids = write(path, nodes, edges, segs)
    return path, [ids[2 * i if two_way else i] for i in range(n_nodes - 1)]


def star(path, lat=40.0, lon=0.0, n_spokes=200, length_m=90.0):
    """A hub with n_spokes two-way straight spokes of length_m, evenly spread
    in bearing: 2 x n_spokes directed edges within length_m of the hub (the
    dense-intersection case past the LDS candidate tier's MAX_HITS).  Each
    outbound spoke is its own level-0 segment (id (i + 1) << 3); inbound
    spokes carry none.  Returns (path, outbound edge ids, inbound edge ids)."""
    ls = MPD * math.cos(math.radians(lat))
    nodes = [(lat, lon)]
    edges, segs = [], []
    for i in range(n_spokes):
        a = 2.0 * math.pi * i / n_spokes
        nodes.append((lat + length_m * math.cos(a) / MPD, lon + length_m * math.sin(a) / ls))
        segs.append(((i + 1) << 3, None))
        edges.append(dict(**{"from": 0, "to": i + 1}, way=5000 + i, seg=i, seg_pos=0, flags=SEG_BEGIN | SEG_END,
                          level=0))
        edges.append(dict(**{"from": i + 1, "to": 0}, way=5000 + i, seg=-1, level=0))
    ids = write(path, nodes, edges, segs)
    return path, [ids[2 * i] for i in range(n_spokes)], [ids[2 * i + 1] for i in range(n_spokes)]
