"""Step timeline from a rocprofv3 kernel trace of bench.py: per k_gc_roundtrip
launch, the GPU front before it (first kernel after the previous launch's
last harvest kernel -> the launch's start), the launch, and the tail after it
(the launch's end -> the last kernel before the next front), with the kernel
time by name in each window.  Usage: step_timeline.py kernel_trace.csv"""
import collections
import csv
import sys


def main(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    launches = [i for i, r in enumerate(rows) if "k_gc_roundtrip" in r[2]]
    print("%d kernels, %d k_gc_roundtrip launches" % (len(rows), len(launches)))
    prev_end_idx = 0
    for n, i in enumerate(launches):
        s, e, _ = rows[i]
        # the front: kernels that start after the previous launch ended (+ its tail) and before this start
        pe = rows[launches[n - 1]][1] if n else None
        front = [r for r in rows[prev_end_idx:i] if (pe is None or r[0] >= pe)]
        # the tail: kernels starting after this launch's end, up to the next launch's front (a gap > 50 ms)
        tail = []
        j = i + 1
        last = e
        while j < len(rows) and (j not in launches):
            r = rows[j]
            if r[0] >= e:
                if r[0] - last > 50e6:
                    break
                tail.append(r)
                last = max(last, r[1])
            j += 1
        prev_end_idx = j
        def by_name(rs):
            d = collections.defaultdict(float)
            for a, b, nm in rs:
                d[nm.split("(")[0][-48:]] += (b - a) * 1e-6
            return sorted(d.items(), key=lambda x: -x[1])[:8]
        if front:
            print("launch %d: front %.1f ms (first kernel -> launch start; %d kernels, busy %.1f ms)"
                  % (n, (s - front[0][0]) * 1e-6, len(front), sum((b - a) for a, b, _ in front) * 1e-6))
            for nm, t in by_name(front):
                print("    %8.1f ms  %s" % (t, nm))
        print("launch %d: %.1f ms" % (n, (e - s) * 1e-6))
        if tail:
            print("launch %d: tail %.1f ms (launch end -> last kernel end; %d kernels)" % (n, (last - e) * 1e-6, len(tail)))
            for nm, t in by_name(tail):
                print("    %8.1f ms  %s" % (t, nm))


if __name__ == "__main__":
    main(sys.argv[1])
