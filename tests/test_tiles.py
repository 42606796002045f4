"""Tile-hierarchy math (reporter_amd/csrc/tiles.cpp) against the reference's
own py/get_tiles.py, recorded in tests/golden/tile_cases.json by
tests/golden/make_tile_golden.py.  CPU only."""
import ctypes as C
import json
import os

import numpy as np

from reporter_amd import synth
from reporter_amd._lib import lib, take

with open(os.path.join(os.path.dirname(__file__), "golden", "tile_cases.json")) as f:
    CASES = json.load(f)


def _file(tid, level, suffix=b"gph"):
    buf = C.create_string_buffer(64)
    assert lib().otm_tile_file(tid, level, suffix, buf, 64) == 0
    return buf.value.decode()


def test_tile_ids_match_get_tiles():
    for c in CASES["ids"]:
        assert lib().otm_tile_id(c["level"], c["lat"], c["lon"]) == c["id"], c
    # Row/Col out of the world bbox: -1 (no id)
    rows = {(c["level"], c["lat"]): c["row"] for c in CASES["rows"]}
    for (level, lat), row in rows.items():
        if row < 0:
            assert lib().otm_tile_id(level, lat, 0.0) == -1


def test_tile_files_match_get_tiles():
    for c in CASES["files"]:
        assert _file(c["id"], c["level"]) == c["file"], c


def test_bbox_listing_matches_get_tiles():
    for c in CASES["bbox"]:
        x0, y0, x1, y1 = (float(v) for v in c["bbox"].split(","))
        out, n = C.c_void_p(), C.c_size_t()
        assert lib().otm_tile_files_bbox(x0, y0, x1, y1, b"gph", C.byref(out), C.byref(n)) == 0
        got = take(out, n.value).decode().split()
        assert sorted(got) == c["files"], c["bbox"]


def test_synthetic_segment_ids_carry_their_tile(small_graph):
    """OSMLR ids of the synthetic graph: level in bits 0-2, the tile id of the
    segment's first shape point (at its level) in bits 3-24 -- the tile math
    above, as py/reporter_service.py:154 reads the level back."""
    ids = synth.segment_ids(small_graph)
    lv = ids & np.uint64(7)
    tiles = (ids >> np.uint64(3)) & np.uint64((1 << 22) - 1)
    assert set(lv.tolist()) <= {0, 1, 2}
    # the extract is 5 x 5 km around (37.98, 23.72): one tile per level
    for level in (0, 1, 2):
        want = lib().otm_tile_id(level, 37.98, 23.72)
        nc = (90, 360, 1440)[level]
        got = set(tiles[lv == level].tolist())
        assert got <= {want + dr * nc + dc for dr in (-1, 0, 1) for dc in (-1, 0, 1)}, (level, got, want)
