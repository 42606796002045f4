"""GPU busy share from a rocprofv3 kernel trace of a bench run with batches in
flight: the union of kernel intervals over the span of the last N k_columns
launches (the timed steps), and the share of time with 1, 2, 3+ kernels
running.  Usage: timeline_busy.py run_kernel_trace.csv [n_steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
cols = [s for s, e, k in iv if "k_columns" in k]
t0, t1 = cols[-n], cols[-1]
ev = []
for s, e, k in iv:
    if e <= t0 or s >= t1:
        continue
    ev.append((max(s, t0), 1))
    ev.append((min(e, t1), -1))
ev.sort()
cur, last, acc = 0, t0, {}
for t, d in ev:
    acc[cur] = acc.get(cur, 0) + (t - last)
    cur += d
    last = t
acc[cur] = acc.get(cur, 0) + (t1 - last)
span = t1 - t0
print("span %.3f ms over %d steps (%.3f ms/step)" % (span / 1e6, n - 1, span / 1e6 / (n - 1)))
for k in sorted(acc):
    print("  %d kernels running: %.1f %%" % (k, 100.0 * acc[k] / span))
