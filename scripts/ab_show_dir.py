"""Summarise one scripts/ab_env_fast.sh output directory: python scripts/ab_show_dir.py gpurun_out/<tag>"""
import glob
import json
import os
import sys

d0 = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d0, "run*.json"))):
    run = os.path.basename(f).split(".")[0]
    env = open(os.path.join(d0, run + ".env")).read().strip() or "(defaults)"
    try:
        d = json.load(open(f))
    except Exception:  # noqa: BLE001
        print("%-34s unreadable" % env)
        continue
    k = d["kernel_ms"]
    top = sorted(k.items(), key=lambda x: -x[1])[:4]
    print("%-34s %-4s %8.1fM pts/s  %.3f ms  same=%s  %s" % (
        env, os.path.basename(f).split(".")[1], d["value"] / 1e6, d["ms_per_step"],
        (d.get("agreement") or {}).get("all_outputs_bit_identical"), " ".join("%s=%.3f" % t for t in top)))
