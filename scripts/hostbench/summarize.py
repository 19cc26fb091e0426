#!/usr/bin/env python3
"""summarize.py LOG -- min / median encode and decode ms per binary of an ab.sh log."""
import collections
import re
import sys

d = collections.defaultdict(lambda: ([], []))
cur = None
for line in open(sys.argv[1]):
    m = re.match(r'== (\S+) round', line)
    if m:
        cur = m.group(1)
        continue
    m = re.match(r'len \d+ enc ([\d.]+) dec ([\d.]+)', line)
    if m:
        d[cur][0].append(float(m.group(1)))
        d[cur][1].append(float(m.group(2)))
for k, (e, dd) in d.items():
    print("%-10s enc min %.1f med %.1f   dec min %.1f med %.1f" % (k, min(e), sorted(e)[len(e) // 2], min(dd), sorted(dd)[len(dd) // 2]))
