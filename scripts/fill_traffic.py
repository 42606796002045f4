"""Put a PMC summary's HBM traffic into a bench line's roofline after the run, with
bench.py's own formulas, when the run's summary could not be matched to the kernel
name at run time (round 4: the template instance k_cand_lane<false> before
scripts/pmc_summary.py aliased it).  The counters are the same box run's.
  python scripts/fill_traffic.py <bench.json> <pmc_traffic.json>"""
import json
import os
import sys

HBM_PEAK_GBS = 8000.0
bpath, tpath = sys.argv[1], sys.argv[2]
d = json.load(open(bpath))
tj = json.load(open(tpath))
r = d["roofline"]
k = r["kernel"]
traffic = tj["kernels"][k]["hbm_bytes_per_launch"]
sec = r["launch_ms"] * 1e-3
own = r.get("algorithmic_bytes_per_launch")
r["traffic"] = traffic
r["traffic_source"] = os.path.relpath(tpath)
r["frac_counter"] = traffic / sec / 1e9 / HBM_PEAK_GBS
r["traffic_correction"] = tj.get("correction")
r["traffic_over_algorithmic"] = traffic / own if own else None
r["traffic_note"] = "filled after the run by scripts/fill_traffic.py from the same run's PMC passes"
json.dump(d, open(bpath, "w"))
print(k, traffic, r["traffic_over_algorithmic"])
