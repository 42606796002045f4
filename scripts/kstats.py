"""Print a rocprofv3 kernel_stats.csv compactly: short name, calls, avg / max us."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("otm::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:44]
    print("%-44s calls=%-5s avg_us=%9.1f max_us=%9.1f" % (n, r["Calls"], float(r["AverageNs"]) / 1e3,
                                                        float(r["MaxNs"]) / 1e3))
