#!/usr/bin/env python3
"""kbench_batch.py -- GPU stages of ric_batch alone (ric_batch_diag_gpu):
per-level per-frame times of the batched fused forward levels and inverse
levels at C3 (or --w/--h), against the SURVEY.md §8(d) byte model.

    python scripts/kbench_batch.py [--slots 16] [--iters 10] [--w 7680 --h 4320]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rududu-image-codec_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--w", type=int, default=7680)
    ap.add_argument("--h", type=int, default=4320)
    ap.add_argument("--q", type=int, default=9)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    import ric_amd
    from bench import wavelet_bytes, HBM_PEAK_GBS
    # device memory from the library itself (no second HIP runtime in the process)
    frames = [ric_amd.DeviceArray.from_numpy(ric_amd.synth(a.w, a.h, 1, f)) for f in range(a.slots)]
    outs = [f.empty_like() for f in frames]
    b = ric_amd.Batch(a.w, a.h, 1, slots=a.slots, threads=1)
    b.diag_gpu(frames, a.q, 0, 2, outs)           # warm-up (argument arrays uploaded)
    b.prof_enable(True)
    b.diag_gpu(frames, a.q, 0, a.iters, outs)
    p = b.prof_read()
    bm = wavelet_bytes(a.w, a.h)
    nl = len(bm["dwt"])
    fwd = [p["fwd_l%d" % l][0] / p["fwd_l%d" % l][1] * 1e3 for l in range(nl)]
    inv = [p["inv_l%d" % l][0] / p["inv_l%d" % l][1] * 1e3 for l in range(nl)]
    enc_b = sum(bm["dwt"]) + sum(bm["quant"]) + bm["ll"]
    dec_b = sum(bm["dwt"]) + sum(bm["deq"])
    out = {"tag": a.tag, "env": {k: v for k, v in os.environ.items() if k.startswith("RIC_")}, "slots": a.slots,
           "fwd_us": [round(x, 2) for x in fwd], "inv_us": [round(x, 2) for x in inv],
           "fwd_total_us": round(sum(fwd), 2), "inv_total_us": round(sum(inv), 2),
           "enc_frac": round(enc_b / (sum(fwd) * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
           "dec_frac": round(dec_b / (sum(inv) * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
           "l0_frac": round((bm["dwt"][0] + bm["quant"][0]) / (fwd[0] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
           "pix_in_us": round(p["pix_in"][0] / p["pix_in"][1] * 1e3, 2) if p["pix_in"][1] else 0.0,
           "pix_out_us": round(p["pix_out"][0] / p["pix_out"][1] * 1e3, 2),
           "d2h_us": round(p["d2h"][0] / p["d2h"][1] * 1e3, 1), "h2d_us": round(p["h2d"][0] / p["h2d"][1] * 1e3, 1),
           "compact_us": round(p["compact"][0] / p["compact"][1] * 1e3, 2) if p["compact"][1] else None,
           "dexp_us": round(p["dcmp_expand"][0] / p["dcmp_expand"][1] * 1e3, 2) if p["dcmp_expand"][1] else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
