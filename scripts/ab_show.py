import glob, json, sys
names = sys.argv[1:] or ["k_cand_lane", "k_trans_sub", "k_route_index"]
for f in sorted(glob.glob("gpurun_out/ab/run*.json")):
    try:
        b = json.loads(open(f).read())
    except Exception as e:
        print(f, "ERR", e); continue
    env = open(f.replace(".json", ".env")).read().strip()
    k = b["kernel_ms"]
    print("%-40s ms %.3f  %s" % (env, b["ms_per_step"], " ".join("%s=%.3f" % (n, k.get(n, -1)) for n in names)))
