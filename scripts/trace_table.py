#!/usr/bin/env python3
"""trace_table.py DIR [PATTERN] -- median duration (us) per (kernel, grid) of a
rocprofv3 --kernel-trace csv directory, largest grid first."""
import csv, os, statistics, sys
d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
per = {}
for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
    n = r["Kernel_Name"].replace("void ric::(anonymous namespace)::", "").replace("ric::(anonymous namespace)::", "")
    n = n[:n.find("(")] if "(" in n else n
    if pat not in n:
        continue
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    per.setdefault((n, g), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
for (n, g), v in sorted(per.items(), key=lambda kv: (kv[0][0].split("<")[0], -kv[0][1])):
    med = statistics.median(v)
    tot += med
    print("%-42s %9d %8.2f us  (n=%d)" % (n[:42], g, med, len(v)))
print("sum of medians: %.2f us" % tot)
