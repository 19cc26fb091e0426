#!/usr/bin/env python3
"""pmc_table.py DIR... -- mean of each PMC counter per kernel name over the
counter_collection.csv files of rocprofv3 --pmc passes (scripts/pmc_sweep.sh)."""
import collections
import csv
import glob
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("void ric::(anonymous namespace)::", "")[:48]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, ctrs in sorted(acc.items()):
    print(name)
    for c, v in sorted(ctrs.items()):
        print("   %-28s %14.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
