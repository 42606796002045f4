#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (scripts/pmc.sh) into per-kernel averages.

Usage: pmc_summary.py <pmc_dir> [tag] [kernel_stats.csv]
With a kernel-trace stats CSV of the same command, each kernel also gets its
achieved HBM GB/s (PMC bytes / average duration) and fraction of 8 TB/s.
LDS bank-conflict rate = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.

hbm_bytes_per_launch = 32 x (TCC_EA0_RDREQ_DRAM_32B + TCC_EA0_WRREQ_WRITE_DRAM_32B
+ TCC_EA0_WRREQ_ATOMIC_DRAM_32B): the DRAM-destined requests in 32-byte units
(rocprofv3 -L on gfx950: "1 64-byte request will be counted to 2, 128-byte as
4"), so every access width is weighted by its real request size -- the
calibration MI355X_MICROARCH.md §HBM asks for instead of its x2 for wide
streaming reads.  (Like FETCH_SIZE, these are memory-side requests;
Infinity-Cache hits are not excluded.)  The FETCH_SIZE x 2 + WRITE_SIZE figure
of round 1 is kept as fetch_x2_write_bytes, and the request-size mix
(TCC_EA0_RDREQ_32B / 64B / 128B of TCC_EA0_RDREQ) shows what the kernel's
gathers cost.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace("otm::(anonymous namespace)::", "").split("(")[0]
    n = n.replace("void ", "").strip()
    if n.startswith("k_segments<128"):
        return "k_segments"  # the small LDS plan (its traversal count is a build knob)
    if n.startswith("k_segments<256"):
        return "k_segments_large"
    alias = {"k_trans_lane<32>": "k_trans_lane", "k_transitions<false>": "k_transitions",
             "k_transitions<true>": "k_transitions_big", "k_route_lane<24>": "k_route_lane",
             "k_route<false>": "k_route", "k_route<true>": "k_route_big",
             "k_transitions<0>": "k_transitions", "k_transitions<1>": "k_transitions_big",
             "k_transitions<2>": "k_transitions_huge", "k_route<0>": "k_route", "k_route<1>": "k_route_big",
             "k_route<2>": "k_route_huge", "k_segments<true>": "k_segments",
             "k_segments<128, 256>": "k_segments", "k_segments<256, 512>": "k_segments_large",
             # the transition index tier's launch slot (otm_kernel_name) runs one of these forms
             "k_trans_sub<4, false>": "k_trans_sub", "k_trans_sub<8, false>": "k_trans_sub", "k_trans_sub<16, false>": "k_trans_sub",
             "k_trans_sub<32, false>": "k_trans_sub", "k_trans_sub<64, false>": "k_trans_sub",
             "k_trans_sub<16, true>": "k_trans_wide",
             # the candidate lane tier: uncounted / counted instances
             "k_cand_lane<false>": "k_cand_lane", "k_cand_lane<true>": "k_cand_lane"}
    return alias.get(n, n)


def durations(stats_csv):
    """Average kernel durations (ns) from a rocprofv3 --stats kernel_stats.csv."""
    out = {}
    for r in csv.DictReader(open(stats_csv)):
        out[short(r["Name"])] = float(r["AverageNs"])
    return out


def main():
    root, tag = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "latest"
    dur = durations(sys.argv[3]) if len(sys.argv) > 3 and os.path.exists(sys.argv[3]) else {}
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
    out = {"tag": tag, "note": "per-launch means over the profiled dispatches",
           "correction": "hbm_bytes = 32 B x size-weighted DRAM read + write + atomic requests (no FETCH_SIZE factor)",
           "kernels": {}}
    for k, cs in sorted(vals.items()):
        d = {cn: sum(v) / len(v) for cn, v in cs.items()}
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["fetch_x2_write_bytes"] = (2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
        dram = [d.get(c) for c in ("TCC_EA0_RDREQ_DRAM_32B_sum", "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum",
                                   "TCC_EA0_WRREQ_ATOMIC_DRAM_32B_sum")]
        if all(v is not None for v in dram):
            d["hbm_read_bytes"] = 32.0 * dram[0]
            d["hbm_write_bytes"] = 32.0 * (dram[1] + dram[2])
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
        if d.get("TCC_EA0_RDREQ_sum"):
            n = d["TCC_EA0_RDREQ_sum"]
            d["read_request_mix"] = {"32B": d.get("TCC_EA0_RDREQ_32B_sum", 0.0) / n,
                                     "64B": d.get("TCC_EA0_RDREQ_64B_sum", 0.0) / n,
                                     "128B": d.get("TCC_EA0_RDREQ_128B_sum", 0.0) / n}
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and d["TCC_HIT_sum"] + d["TCC_MISS_sum"] > 0:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        if d.get("SQ_LDS_IDX_ACTIVE"):
            # share of LDS-active cycles lost to bank conflicts
            d["lds_bank_conflict_rate"] = d.get("SQ_LDS_BANK_CONFLICT", 0.0) / d["SQ_LDS_IDX_ACTIVE"]
        if k in dur and "hbm_bytes_per_launch" in d and dur[k] > 0:
            d["avg_duration_ns"] = dur[k]
            d["hbm_GB_per_s"] = d["hbm_bytes_per_launch"] / dur[k]
            d["hbm_frac_of_8TBps"] = d["hbm_GB_per_s"] / 8000.0
        out["kernels"][k] = d
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
