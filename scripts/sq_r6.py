#!/usr/bin/env python3
"""sq_r6.py TAG RUN "WHAT" -- adds a run to profiles/r06_stream_coder_sq.json
(the issue counters bench.py reports as stream_coder.issue) from a
scripts/gpu_sq.sh TAG run over one serving step (bench.py --steps 1 --warmup 0
--n-host 0: one k_gc_roundtrip launch of 3072 C3 streams), and makes it the
default run.  Fields as scripts/sq_head.py: SQ_INSTS_* in millions of
wave-instructions per stream, clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time,
SALU per CU per cycle, (SALU + VALU) per SIMD per 4-cycle issue turn,
SQ_WAIT_ANY / SQ_WAVE_CYCLES."""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, name, what = sys.argv[1:4]
    p = glob.glob(os.path.join(REPO, "gpurun_out", tag + "_sq", "**", "*counter_collection.csv"), recursive=True)[0]
    d = {}
    for r in csv.DictReader(open(p)):
        if "k_gc_roundtrip" not in r["Kernel_Name"]:
            continue
        e = d.setdefault(r["Dispatch_Id"], {"grid": int(r["Grid_Size"]),
                                            "s": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    (e,) = d.values()
    n = e["grid"] // 64
    cyc = e["GRBM_GUI_ACTIVE"] / 8
    run = {"what": what, "kernel_s": round(e["s"], 3), "streams": n}
    for k in ("SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS"):
        run[k] = round(e[k] / n / 1e6, 2)
    run["salu_share"] = round(e["SQ_INSTS_SALU"] / (e["SQ_INSTS_SALU"] + e["SQ_INSTS_VALU"]), 3)
    run["clock_ghz"] = round(cyc / e["s"] / 1e9, 3)
    run["salu_per_cu_cycle"] = round(e["SQ_INSTS_SALU"] / 256 / cyc, 3)
    run["instr_per_simd_per_4_cycles"] = round((e["SQ_INSTS_SALU"] + e["SQ_INSTS_VALU"]) / 1024 / (cyc / 4), 3)
    run["wait_frac"] = round(e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"], 3)
    run["units"] = "SQ_INSTS_* in millions of wave-instructions per stream; clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time"
    f = os.path.join(REPO, "profiles", "r06_stream_coder_sq.json")
    out = json.load(open(f))
    out["runs"][name] = run
    out["default_run"] = name
    out["source"] = ("scripts/gpu_sq.sh %s (rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS "
                     "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT over bench.py "
                     "--steps 1 --warmup 0 --n-host 0)" % tag)
    json.dump(out, open(f, "w"), indent=1)
    print(json.dumps(run, indent=1))


if __name__ == "__main__":
    main()
