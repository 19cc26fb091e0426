#!/usr/bin/env python3
"""salu_summary.py OUT.json LABEL=counter_collection.csv ... -- the GPU stream
coder's issue fractions from rocprofv3 --pmc passes over scripts/gc_probe.py:
per dispatch of k_gc_encode / k_gc_decode, SQ_INSTS_SALU (and every
instruction type) per CU per cycle, cycles = GRBM_GUI_ACTIVE / 8 (the counter
sums the 8 XCDs), 256 CUs; SQ_WAIT_ANY / SQ_WAVE_CYCLES = the waves' waiting
share.  One scalar unit per CU issues at most one SALU instruction a cycle."""
import collections
import csv
import json
import sys

CUS = 256


def summarise(path):
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if "k_gc_" not in r["Kernel_Name"]:
            continue
        e = d[r["Dispatch_Id"]]
        e[r["Counter_Name"]] = float(r["Counter_Value"])
        e["kernel"] = "k_gc_encode" if "encode" in r["Kernel_Name"] else "k_gc_decode"
        e["grid"] = int(r["Grid_Size"])
        e["s"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = collections.defaultdict(list)
    for e in d.values():
        cyc = e["GRBM_GUI_ACTIVE"] / 8
        ins = sum(e.get(k, 0) for k in ("SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"))
        out[e["kernel"]].append({"streams": e["grid"] // 64, "s": round(e["s"], 4), "clock_ghz": round(cyc / e["s"] / 1e9, 2),
                                 "salu_frac": round(e["SQ_INSTS_SALU"] / CUS / cyc, 4),
                                 "issue_frac_all": round(ins / CUS / cyc, 4),
                                 "wait_frac": round(e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"], 4),
                                 "salu_instructions": e["SQ_INSTS_SALU"], "valu_instructions": e["SQ_INSTS_VALU"]})
    return out


def main():
    res = {"method": __doc__.strip().splitlines()[0], "runs": {}}
    for arg in sys.argv[2:]:
        label, path = arg.split("=", 1)
        res["runs"][label] = summarise(path)
    json.dump(res, open(sys.argv[1], "w"), indent=1)
    for label, r in res["runs"].items():
        for k, v in r.items():
            print(label, k, [(x["salu_frac"], x["issue_frac_all"], x["wait_frac"]) for x in v])


if __name__ == "__main__":
    main()
