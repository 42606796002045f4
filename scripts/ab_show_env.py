"""Summarise gpurun_out/abe (scripts/ab_env_configs.sh)."""
import glob
import json
import os

for f in sorted(glob.glob("gpurun_out/abe/run*.json")):
    d = json.load(open(f))
    run = os.path.basename(f).split(".")[0]
    env = open("gpurun_out/abe/%s.env" % run).read().strip() or "(defaults)"
    k = d["kernel_ms"]
    top = sorted(k.items(), key=lambda x: -x[1])[:4]
    print("%-28s %-4s %8.1fM pts/s  same=%s  %s" % (env, os.path.basename(f).split(".")[1], d["value"] / 1e6,
          (d.get("agreement") or {}).get("all_outputs_bit_identical"), " ".join("%s=%.3f" % t for t in top)))
