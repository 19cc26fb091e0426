#!/usr/bin/env python3
"""pmc_levels.py TAG -- profiles/pmc_fwd_levels_batch.json from a
scripts/r5_pmc_levels.sh run: the HBM bytes per frame of the whole 5-level
forward encode (every k_fwdq_* dispatch of kbench_batch.py's groups of 16 C3
frames), FETCH_SIZE x2 (the gfx950 correction, MI355X_MICROARCH.md HBM
section) + WRITE_SIZE, both KiB; per level as well."""
import csv
import glob
import json
import os
import re
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def load(tag, c):
    p = glob.glob(os.path.join(REPO, "gpurun_out", "%s_pmc_%s" % (tag, c), "**", "*counter_collection.csv"), recursive=True)
    rows = list(csv.DictReader(open(p[0])))
    return [r for r in rows if r["Counter_Name"] == c and "k_fwdq" in r["Kernel_Name"]]


def main():
    tag = sys.argv[1]
    from bench import wavelet_bytes
    slots = 16
    out = {"W": 7680, "H": 4320, "frames_per_launch": slots, "levels": []}
    per = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rs = load(tag, c)
        # dispatch order: level 0..4 per group (diag_gpu), groups repeat
        by = {}
        for r in rs:
            by.setdefault(re.search(r"(k_fwdq\w*(<[^(]*>)?)", r["Kernel_Name"]).group(1), []).append(float(r["Counter_Value"]))
        per[c] = by
    names = list(per["FETCH_SIZE"].keys())
    bm = wavelet_bytes(7680, 4320)
    # groups of frames: the level-0 kernel runs once per group (levels 3 and 4
    # may share a kernel name: their dispatches are summed per group)
    ngroups = min(len(v) for k, v in per["FETCH_SIZE"].items() if k.startswith("k_fwdq_pc_z8") or k == "k_fwdq_pc_z<false, false>")
    tot = 0.0
    for n in names:
        f = sum(per["FETCH_SIZE"][n]) * 2 * 1024 / ngroups
        w = sum(per["WRITE_SIZE"][n]) * 1024 / ngroups
        out["levels"].append({"kernel": n, "dispatches_per_group": len(per["FETCH_SIZE"][n]) / ngroups,
                              "hbm_bytes_per_frame": round((f + w) / slots)})
        tot += (f + w) / slots
    out["hbm_bytes_per_frame_all_levels"] = round(tot)
    out["algorithmic_bytes_per_frame"] = sum(bm["dwt"]) + sum(bm["quant"]) + bm["ll"]
    out["correction"] = "FETCH_SIZE x2 (gfx950), WRITE_SIZE as is; KiB -> B; every dispatch summed, divided by the groups (level-0 dispatches) and the frames per group"
    out["source"] = ("round 5: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, over scripts/kbench_batch.py "
                     "--iters 3 (ric_batch_diag_gpu: the 5 forward levels of 16 C3 frames alone, the level kernels' "
                     "alone forms)")
    json.dump(out, open(os.path.join(REPO, "profiles", "pmc_fwd_levels_batch.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
