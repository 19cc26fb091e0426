#!/usr/bin/env python3
"""pmc_table.py DIR... -- mean of each PMC counter per (kernel name, grid size)
over the counter_collection.csv files of rocprofv3 --pmc passes
(scripts/pmc_sweep.sh)."""
import collections
import csv
import glob
import os
import sys


def grid(r):
    if "Grid_Size_X" in r:
        return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    return int(r.get("Grid_Size", 0))


acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("void ", "").replace("ric::(anonymous namespace)::", "")
            name = name[:name.find("(")] if "(" in name else name
            acc[(name[:40], grid(r))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (name, g), ctrs in sorted(acc.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
    print("%s grid=%d" % (name, g))
    for c, v in sorted(ctrs.items()):
        print("   %-28s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
