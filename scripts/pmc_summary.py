#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (scripts/pmc.sh) into per-kernel averages.

hbm_bytes_per_launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
streaming read, so the read side is doubled (an upper bound for narrower
access shapes, which the guide leaves uncalibrated).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace("otm::(anonymous namespace)::", "").split("(")[0]
    n = n.replace("void ", "")
    alias = {"k_trans_lane<32>": "k_trans_lane", "k_transitions<false>": "k_transitions",
             "k_transitions<true>": "k_transitions_big", "k_route_lane<24>": "k_route_lane",
             "k_route<false>": "k_route", "k_route<true>": "k_route_big", "k_segments<true>": "k_segments",
             "k_segments<128, 256>": "k_segments", "k_segments<256, 512>": "k_segments_large",
             # the transition index tier's launch slot (otm_kernel_name) runs one of these forms
             "k_trans_sub<16>": "k_trans_index", "k_trans_sub<32>": "k_trans_index"}
    return alias.get(n, n)


def main():
    root, tag = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "latest"
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (disp, cn), v in per.items():
            vals[names[disp]][cn].append(v)
    out = {"tag": tag, "note": "per-launch means over the profiled dispatches; FETCH_SIZE doubled (gfx950)",
           "kernels": {}}
    for k, cs in sorted(vals.items()):
        d = {cn: sum(v) / len(v) for cn, v in cs.items()}
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and d["TCC_HIT_sum"] + d["TCC_MISS_sum"] > 0:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        out["kernels"][k] = d
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
