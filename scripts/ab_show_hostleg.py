"""Summarise gpurun_out/abh/*.json (scripts/ab_hostleg.sh)."""
import glob
import json
import os

for f in sorted(glob.glob("gpurun_out/abh/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    h = d.get("host_inclusive") or {}
    print("%-14s device %7.1fM pts/s (%.3f ms)   host-inclusive %7.1fM pts/s (%.3f ms)" % (
        os.path.basename(f)[:-5], d["value"] / 1e6, d["ms_per_step"], h.get("value", 0) / 1e6, h.get("ms_per_step", 0)))
