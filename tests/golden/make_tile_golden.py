#!/usr/bin/env python3
"""Tile-hierarchy fixtures from the REFERENCE itself (build container only).

TEST INFRASTRUCTURE, like make_golden.py: it runs /root/reference/py/get_tiles.py
(read-only, never copied) and records its input/output behaviour as JSON data
in tests/golden/tile_cases.json:

  rows/cols   Tiles.Row / Tiles.Col per level (py/get_tiles.py:51-72) at sample
              latitudes / longitudes, bounds and tile edges included
  ids         tile id = Row * ncolumns + Col (the main loop, :159-168)
  files       Tiles.GetFile(tile_id, level) (:82-102) with suffix "gph"
  bbox        the tile files the script lists for a bounding box (-b/-s,
              :130-172, run as __main__ with its stdout captured), per level

get_tiles.py is Python 2: it is exec'd in memory with `long` bound to int (its
only Python-2-only name; its integer `/=` in Digits gives the same digit
count on floats).  Bytecode writing is off; nothing is written under
/root/reference.  Only the JSON is committed.
"""
import sys
sys.dont_write_bytecode = True
import contextlib
import io
import json
import os
import warnings

warnings.simplefilter("ignore")
REF = "/root/reference/py/get_tiles.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tile_cases.json")


def load(argv=None, main=False):
    src = open(REF).read()
    ns = {"__name__": "__main__" if main else "ref_get_tiles", "long": int}
    old = sys.argv
    sys.argv = ["get_tiles.py"] + (argv or [])
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            exec(compile(src, "get_tiles.py", "exec"), ns)
    finally:
        sys.argv = old
    return ns, buf.getvalue()


def main():
    ns, _ = load()
    th = ns["TileHierarchy"]()
    ns["suffix"] = "gph"
    lats = [-90.0, -89.999, -45.5, -0.25, -0.0001, 0.0, 0.1, 0.25, 14.5, 37.98, 37.999999, 38.0, 60.75, 89.99, 90.0,
            -90.5, 90.5]
    lons = [-180.0, -179.75, -120.2, -0.3, -0.0001, 0.0, 0.3, 23.72, 121.0, 121.021019, 179.75, 179.9, 180.0,
            -180.5, 180.5]
    out = {"rows": [], "cols": [], "ids": [], "files": [], "bbox": []}
    for level in (0, 1, 2):
        t = th.levels[level]
        for y in lats:
            out["rows"].append({"level": level, "lat": y, "row": t.Row(y)})
        for x in lons:
            out["cols"].append({"level": level, "lon": x, "col": t.Col(x)})
        for y in lats:
            for x in lons:
                r, c = t.Row(y), t.Col(x)
                if r < 0 or c < 0:
                    continue
                out["ids"].append({"level": level, "lat": y, "lon": x, "id": r * t.ncolumns + c})
        for tid in (0, 1, 7, 1000, 1234, t.max_tile_id // 2, t.max_tile_id):
            out["files"].append({"level": level, "id": tid, "file": t.GetFile(tid, level)})
    for bb in ("121.0,14.5,121.1,14.6", "23.6,37.9,23.8,38.05", "-74.251961,40.512764,-73.755405,40.903125",
               "179.9,10.0,-179.9,10.3"):
        _, text = load(["-b", bb, "-s", "gph"], main=True)
        out["bbox"].append({"bbox": bb, "files": sorted(text.split())})
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("wrote %s: %d rows, %d cols, %d ids, %d files, %d bboxes" %
          (OUT, len(out["rows"]), len(out["cols"]), len(out["ids"]), len(out["files"]), len(out["bbox"])))


if __name__ == "__main__":
    main()
