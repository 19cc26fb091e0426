#!/usr/bin/env python3
"""kstats.py DIR... -- per-kernel average duration table from rocprofv3 --stats CSVs."""
import csv
import os
import sys

for d in sys.argv[1:]:
    f = os.path.join(d, "run_kernel_stats.csv")
    print("==", d)
    for r in csv.DictReader(open(f)):
        name = r["Name"].replace("void ric::(anonymous namespace)::", "").replace("ric::(anonymous namespace)::", "")
        print("%10.2f us %5s calls  %s" % (float(r["AverageNs"]) / 1e3, r["Calls"], name[:90]))
