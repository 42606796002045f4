"""Summarise gpurun_out/abv/*.json (scripts/ab_variants.sh)."""
import glob
import json
import os

for f in sorted(glob.glob("gpurun_out/abv/*.json")):
    try:
        d = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    k = d["kernel_ms"]
    top = sorted(k.items(), key=lambda x: -x[1])[:5]
    print("%-16s %8.1fM pts/s  %.3f ms/step  same=%s  %s" % (
        os.path.basename(f)[:-5], d["value"] / 1e6, d["ms_per_step"],
        (d.get("agreement") or {}).get("all_outputs_bit_identical"),
        " ".join("%s=%.3f" % t for t in top)))
