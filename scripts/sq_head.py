#!/usr/bin/env python3
"""sq_head.py ISSUE_TAG FETCH_TAG WRITE_TAG -- profiles/r05_stream_coder_sq.json
and profiles/pmc_fwd_l0_batch.json from scripts/gpu_sq.sh runs over one
serving step at HEAD (bench.py --steps 1 --warmup 0 --n-host 0: one
k_gc_roundtrip launch of 3072 C3 streams, 192 level-0 groups of 16 frames).
Coder fields as profiles/r04_stream_coder_sq.json: counters per stream (the
totals over the launch / streams; GRBM summed over the 8 XCDs), clock =
GRBM_GUI_ACTIVE / 8 / kernel time, SALU per CU per cycle, (SALU + VALU) per
SIMD per 4-cycle issue turn, SQ_WAIT_ANY / SQ_WAVE_CYCLES.  Level-0 bytes:
FETCH_SIZE x2 (gfx950) + WRITE_SIZE, KiB -> B, medians over the dispatches."""
import csv
import glob
import json
import os
import re
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(tag):
    p = glob.glob(os.path.join(REPO, "gpurun_out", tag + "_sq", "**", "*counter_collection.csv"), recursive=True)[0]
    return list(csv.DictReader(open(p)))


def main():
    it, ft, wt = sys.argv[1:4]
    d = {}
    for r in rows(it):
        if "k_gc_roundtrip" not in r["Kernel_Name"]:
            continue
        e = d.setdefault(r["Dispatch_Id"], {"grid": int(r["Grid_Size"]),
                                            "s": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    (e,) = d.values()
    n = e["grid"] // 64
    cyc = e["GRBM_GUI_ACTIVE"] / 8
    run = {"what": "round 5 HEAD (88-VGPR coder, UCOND 2, EFIFO 1): one k_gc_roundtrip launch of %d streams, "
                   "three coder waves on every SIMD" % n, "kernel_s": round(e["s"], 2), "streams": n}
    for k in ("GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM",
              "SQ_INSTS_VALU", "SQ_WAIT_ANY", "SQ_WAVES", "SQ_WAVE_CYCLES"):
        if k in e:
            run[k] = round(e[k] / n)
    run["clock_ghz"] = round(cyc / e["s"] / 1e9, 3)
    run["salu_share"] = round(e["SQ_INSTS_SALU"] / (e["SQ_INSTS_SALU"] + e["SQ_INSTS_VALU"]), 3)
    run["instr_per_simd_per_4_cycles"] = round((e["SQ_INSTS_SALU"] + e["SQ_INSTS_VALU"]) / 1024 / (cyc / 4), 3)
    run["salu_per_cu_cycle"] = round(e["SQ_INSTS_SALU"] / 256 / cyc, 3)
    run["wait_frac"] = round(e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"], 3)
    run["salu_plus_valu_per_stream"] = round((e["SQ_INSTS_SALU"] + e["SQ_INSTS_VALU"]) / n)
    prev = json.load(open(os.path.join(REPO, "profiles", "r04_stream_coder_sq.json")))
    out = {"method": prev["method"], "streams": n, "runs": {"r5_head": run,
                                                            "r4z_c3072": prev["runs"]["r4z_c3072"]},
           "default_run": "r5_head",
           "source": "rocprofv3 --pmc (scripts/gpu_sq.sh %s - issue) over one serving step at HEAD; "
                     "r4z_c3072: round 4's for comparison" % it}
    json.dump(out, open(os.path.join(REPO, "profiles", "r05_stream_coder_sq.json"), "w"), indent=1)
    print(json.dumps(run, indent=1))
    # level 0's HBM bytes in the step
    by = {}
    for tag, c in ((ft, "FETCH_SIZE"), (wt, "WRITE_SIZE")):
        for r in rows(tag):
            m = re.search(r"(k_fwdq_pc_z8?<[^(]*>)", r["Kernel_Name"])
            if m and r["Counter_Name"] == c:
                by.setdefault((m.group(1), c), []).append(float(r["Counter_Value"]))
    names = sorted({k[0] for k in by})
    l0 = [k for k in names if k.startswith("k_fwdq_pc_z8")]
    name = l0[0] if l0 else names[0]
    f = by[(name, "FETCH_SIZE")]
    w = by[(name, "WRITE_SIZE")]
    rb = statistics.median(f) * 2 * 1024
    wb = statistics.median(w) * 1024
    frames = 16
    l0j = {"kernel": name + " level 0 (the serving step's form: 8-bit pixels in, level shift fused; bands into the "
                              "scratch arenas, records into the pool)",
           "W": 7680, "H": 4320, "frames_per_launch": frames, "launches": len(f),
           "fetch_size_kib_raw_median": statistics.median(f), "write_size_kib_raw_median": statistics.median(w),
           "read_bytes_corrected": rb, "write_bytes": wb, "hbm_bytes_per_launch": round(rb + wb),
           "hbm_bytes_per_frame": round((rb + wb) / frames),
           "correction": "FETCH_SIZE x2 (gfx950 reports half of a wide coalesced stream, MI355X_MICROARCH.md HBM "
                         "section), WRITE_SIZE as is; KiB -> B",
           "source": "round 5 HEAD: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over one "
                     "serving step (scripts/gpu_sq.sh %s / %s: bench.py --steps 1 --warmup 0 --n-host 0), medians "
                     "over the %d level-0 dispatches (FETCH min/max %.0f/%.0f KiB, WRITE %.0f/%.0f KiB)"
                     % (ft, wt, len(f), min(f), max(f), min(w), max(w))}
    old = json.load(open(os.path.join(REPO, "profiles", "pmc_fwd_l0_batch.json")))
    l0j["previous"] = {"hbm_bytes_per_frame": old["hbm_bytes_per_frame"], "source": old["source"]}
    l0j["algorithmic_bytes_per_frame"] = old.get("algorithmic_bytes_per_frame")
    json.dump(l0j, open(os.path.join(REPO, "profiles", "pmc_fwd_l0_batch.json"), "w"), indent=1)
    print(name, l0j["hbm_bytes_per_frame"], len(f))


if __name__ == "__main__":
    main()
