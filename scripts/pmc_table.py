#!/usr/bin/env python3
"""pmc_table.py TAG -- per-kernel (name, grid) median of every counter in gpurun_out/TAG_p*/"""
import csv, glob, os, statistics, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
tab = {}
for f in sorted(glob.glob(os.path.join(REPO, "gpurun_out", tag + "_p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ric::(anonymous namespace)::", "").split("(")[0]
        if pat not in n:
            continue
        key = (n, int(r.get("Grid_Size", 0)))
        tab.setdefault(key, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for (n, g), cs in sorted(tab.items(), key=lambda kv: -kv[0][1]):
    print("%-40s grid=%-8d " % (n[:40], g) + " ".join("%s=%.4g" % (c, statistics.median(v)) for c, v in sorted(cs.items())))
