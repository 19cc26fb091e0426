#!/usr/bin/env python3
"""batch_prof_summary.py TAG [ROUND] [SLOTS] -- turn scripts/r2_profile.sh output
(merged into gpurun_out/) into committed artefacts:

  profiles/ROUND_TAG_bench_kernel_stats.csv   rocprofv3 --stats of bench.py
  profiles/ROUND_TAG_bench_kernel_medians.txt per kernel and grid: launches,
        median / mean duration, and per frame (÷ frames per launch = grid z)
  profiles/ROUND_TAG_kbench_kernel_medians.txt  the same for kbench_batch.py
  profiles/pmc_fwd_l0_batch.json  HBM traffic of the level-0 batched launch
        (k_fwdq_pc_z, largest grid): FETCH_SIZE x2 (gfx950: half of a wide
        coalesced stream, MI355X_MICROARCH.md) + WRITE_SIZE, KiB -> B, per
        launch and per frame
"""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")


def rows(p):
    with open(p, newline="") as f:
        return list(csv.DictReader(f))


def short(n):
    n = n.replace("ric::(anonymous namespace)::", "").replace("void ", "")
    return n[:n.find("(")] if "(" in n else n


def grid3(r):
    if "Grid_Size_X" in r:
        return int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"])
    return int(r["Grid_Size"]), 1, 1


def medians(trace, dst):
    per = {}
    for r in rows(trace):
        per.setdefault((short(r["Kernel_Name"]), grid3(r)), []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = ["%-52s %-18s %7s %10s %10s %10s" % ("kernel", "grid", "calls", "median_us", "mean_us", "us/frame")]
    for (k, g), v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        z = g[2] if ("_z<" in k or k.endswith("_z")) else 1
        med = statistics.median(v)
        lines.append("%-52s %-18s %7d %10.2f %10.2f %10.2f" % (k, "%dx%dx%d" % g, len(v), med, statistics.mean(v), med / z))
    open(dst, "w").write("\n".join(lines) + "\n")
    return per


def pmc(tag, counter):
    p = os.path.join(OUT, "%s_pmc_%s" % (tag, counter.split("_")[0].lower()), "run_counter_collection.csv")
    rs = [r for r in rows(p) if r["Counter_Name"] == counter and short(r["Kernel_Name"]) == "k_fwdq_pc_z<true>"]
    g = max(int(r["Grid_Size"]) for r in rs)
    sel = [float(r["Counter_Value"]) for r in rs if int(r["Grid_Size"]) == g]
    return statistics.mean(sel), len(sel)


def main():
    tag = sys.argv[1]
    rnd = sys.argv[2] if len(sys.argv) > 2 else "r02"
    slots = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(os.path.join(OUT, tag + "_bkt", "run_kernel_stats.csv"),
                os.path.join(PROF, "%s_%s_bench_kernel_stats.csv" % (rnd, tag)))
    per = medians(os.path.join(OUT, tag + "_bkt", "run_kernel_trace.csv"),
                  os.path.join(PROF, "%s_%s_bench_kernel_medians.txt" % (rnd, tag)))
    medians(os.path.join(OUT, tag + "_kkt", "run_kernel_trace.csv"),
            os.path.join(PROF, "%s_%s_kbench_kernel_medians.txt" % (rnd, tag)))
    l0 = [v for (k, g), v in per.items() if k == "k_fwdq_pc_z<true>"]
    l0 = max(l0, key=len) if l0 else []
    f, nf = pmc(tag, "FETCH_SIZE")
    w, nw = pmc(tag, "WRITE_SIZE")
    rd = f * 1024 * 2
    wr = w * 1024
    out = {"kernel": "k_fwdq_pc_z level 0 (largest-grid launch of the batched fused forward DWT + quantiser)",
           "W": 7680, "H": 4320, "frames_per_launch": slots,
           "fwd_l0_median_us_bench_trace": round(statistics.median(l0), 2) if l0 else None,
           "fetch_size_kib_raw": round(f, 1), "write_size_kib_raw": round(w, 1), "launches": [nf, nw],
           "read_bytes_corrected": rd, "write_bytes": wr,
           "hbm_bytes_per_launch": int(rd + wr), "hbm_bytes_per_frame": int((rd + wr) / slots),
           "correction": "FETCH_SIZE x2 (gfx950 reports half of a wide coalesced stream), WRITE_SIZE as is; KiB -> B",
           "source": "gpurun_out/%s_pmc_{fetch,write}/run_counter_collection.csv (scripts/kbench_batch.py, C3)" % tag}
    json.dump(out, open(os.path.join(PROF, "pmc_fwd_l0_batch.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
