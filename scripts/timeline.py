"""Timeline of a rocprofv3 --kernel-trace --memory-copy-trace run (gpurun_out/<dir>/run_*.csv):
the last `--window` ms, per stream: copies (direction, bytes unknown -> duration) and kernel busy time,
plus how much of the window each resource (H2D, D2H, any kernel) is busy."""
import csv
import sys

d = sys.argv[1]
win_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
K = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
M = list(csv.DictReader(open(d + "/run_memory_copy_trace.csv")))
ev = []
for k in K:
    ev.append(("K", int(k["Stream_Id"]), int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"][:40]))
for m in M:
    ev.append((m["Direction"].replace("MEMORY_COPY_", ""), int(m["Stream_Id"]), int(m["Start_Timestamp"]),
               int(m["End_Timestamp"]), ""))
end = max(e[3] for e in ev)
t0 = end - win_ms * 1e6
ev = [e for e in ev if e[3] > t0]


def busy(kind):
    iv = sorted((max(e[2], t0), e[3]) for e in ev if (e[0] == kind if kind != "K" else e[0] == "K"))
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot / 1e6


print("window %.1f ms: busy H2D %.2f ms, D2H %.2f ms, kernels %.2f ms" %
      (win_ms, busy("HOST_TO_DEVICE"), busy("DEVICE_TO_HOST"), busy("K")))
for kind in ("HOST_TO_DEVICE", "DEVICE_TO_HOST", "DEVICE_TO_DEVICE"):
    ds = sorted(((e[3] - e[2]) / 1e3) for e in ev if e[0] == kind)
    if ds:
        print(kind, "n=%d" % len(ds), "sum %.2f ms" % (sum(ds) / 1e3), "largest (us):", ["%.0f" % x for x in ds[-8:]])
if "-v" in sys.argv:
    for e in sorted(ev, key=lambda e: e[2]):
        print("%9.3f %9.3f s%d %-16s %s" % ((e[2] - t0) / 1e6, (e[3] - e[2]) / 1e6, e[1], e[0], e[4]))
