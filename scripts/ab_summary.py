#!/usr/bin/env python3
"""Summarise an A/B directory of bench lines (gpurun_out/<tag>/bench_*.json):
points/s and the main kernels' HIP-event times, one line per file."""
import glob
import json
import os
import sys

KERNELS = ("k_cand_lane", "k_trans_sub", "k_viterbi", "k_route_index", "k_seg_bound", "scan_seg_bound", "k_segments")


def main():
    d = sys.argv[1]
    for f in sorted(glob.glob(os.path.join(d, "bench_*.json"))):
        try:
            line = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError) as e:
            print(os.path.basename(f), "unreadable:", e)
            continue
        km = line.get("kernel_ms", {})
        print(os.path.basename(f), "%.4fG" % (line["value"] / 1e9),
              " ".join("%s=%.4f" % (k, km[k]) for k in KERNELS if k in km))
    for log in sorted(glob.glob(os.path.join(d, "pytest*.log"))):
        print(os.path.basename(log), open(log).read().strip().splitlines()[-1])


if __name__ == "__main__":
    main()
