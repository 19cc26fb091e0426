#!/usr/bin/env python3
"""pmc_summary.py TAG [ROUND] -- turn a scripts/gpu_profile.sh run (merged back
into gpurun_out/) into the committed profile artefacts:

  profiles/ROUND_TAG_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/ROUND_TAG_kernel_trace_summary.json
        per-kernel-instance durations (level-0 forward DWT picked out by its
        grid size, the largest k_fwd launch)
  profiles/pmc_fwd_l0.json              HBM traffic per level-0 k_fwd launch

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come from
separate passes, both in KiB; on gfx950 FETCH_SIZE reports half the bytes of a
wide coalesced stream, so the read side is doubled (the kernel reads 8 B per
lane per row; the raw values are kept alongside).
"""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def grid(r):
    if "Grid_Size_X" in r:
        return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    return int(r["Grid_Size"])


def fwd_l0(rs):
    """The level-0 launches of the fused forward level kernel (largest grid)."""
    fw = [r for r in rs if "k_fwdq_pc<" in r["Kernel_Name"] or r["Kernel_Name"].startswith("ric::(anonymous namespace)::k_fwdq_pc(")]
    if not fw:
        return []
    g = max(grid(r) for r in fw)
    return [r for r in fw if grid(r) == g]


def counter(tag, name):
    p = os.path.join(REPO, "gpurun_out", "%s_pmc_%s" % (tag, name.split("_")[0].lower()), "run_counter_collection.csv")
    if not os.path.exists(p):
        return None
    rs = [r for r in rows(p) if r["Counter_Name"] == name]
    sel = fwd_l0(rs)
    if not sel:
        return None
    return statistics.mean(float(r["Counter_Value"]) for r in sel), len(sel)


def main():
    tag = sys.argv[1]
    # TAG_kt (kernel trace), TAG_pmc_fetch / TAG_pmc_write (counter passes)
    rnd = sys.argv[2] if len(sys.argv) > 2 else "r01"
    kt = os.path.join(REPO, "gpurun_out", tag + "_kt")
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    out = {}
    st = os.path.join(kt, "run_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, os.path.join(REPO, "profiles", "%s_%s_kernel_stats.csv" % (rnd, tag)))
    tr = os.path.join(kt, "run_kernel_trace.csv")
    if os.path.exists(tr):
        rs = rows(tr)
        per = {}
        for r in rs:
            name = r["Kernel_Name"].replace("ric::(anonymous namespace)::", "").replace("void ", "")
            name = name[:name.rfind("(")] if name.endswith(")") else name
            key = "%s grid=%d" % (name, grid(r))
            per.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        summ = {k: {"calls": len(v), "avg_us": round(statistics.mean(v), 2), "min_us": round(min(v), 2),
                    "max_us": round(max(v), 2)} for k, v in sorted(per.items())}
        l0 = fwd_l0(rs)
        if l0:
            d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in l0]
            out["fwd_l0_avg_us_kernel_trace"] = round(statistics.mean(d), 2)
            out["fwd_l0_launches"] = len(d)
        with open(os.path.join(REPO, "profiles", "%s_%s_kernel_trace_summary.json" % (rnd, tag)), "w") as f:
            json.dump(summ, f, indent=1)
    fe = counter(tag, "FETCH_SIZE")
    wr = counter(tag, "WRITE_SIZE")
    if fe and wr:
        fetch_b = fe[0] * 1024.0
        write_b = wr[0] * 1024.0
        out.update({
            "kernel": "k_fwdq_pc level 0 (largest-grid launch of the fused forward DWT + quantiser)",
            "fetch_size_kib_raw": round(fe[0], 1), "write_size_kib_raw": round(wr[0], 1),
            "launches": [fe[1], wr[1]],
            "read_bytes_corrected": 2 * fetch_b, "write_bytes": write_b,
            "hbm_bytes_per_launch": int(2 * fetch_b + write_b),
            "correction": "FETCH_SIZE x2 (gfx950 reports half of a wide coalesced stream), WRITE_SIZE as is; KiB -> B",
            "source": "gpurun_out/%s_pmc_{fetch,write}/run_counter_collection.csv" % tag,
        })
        with open(os.path.join(REPO, "profiles", "pmc_fwd_l0.json"), "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
