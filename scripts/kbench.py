#!/usr/bin/env python3
"""kbench.py -- uncontended GPU stage timings on one 8K frame (single thread).

  python scripts/kbench.py [--iters N] [--width W --height H] [--codec]

Times the device stages in isolation with the library's HIP-event stage
timers: the fused forward DWT + quantiser + records (ric_transform_quantize;
"fwd_l0" = the level-0 kernel, "fwd" = the whole device encode, "quant" =
nothing unless RIC_NOFUSE=1 splits it off), then, with --codec, one full encode+decode per iteration on a
single codec (stage breakdown incl. the host coder).  Used for kernel tuning
and under rocprofv3; bench.py is the contract benchmark.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rududu-image-codec_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--codec", action="store_true")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    import ric_amd
    W, H = a.width, a.height
    pix = ric_amd.synth(W, H, 1, 0)
    img = torch.from_numpy(((pix[0].astype(np.int16) - 128) << 4)).cuda()
    torch.cuda.synchronize()
    w = ric_amd.Wavelet2D(W, H, 5, 1)
    w.SetWeight(0)
    q, lam = ric_amd.quants(29), ric_amd.quants(22)
    out = {"config": "%dx%d gray 9/7 5 levels, Quant %d lambda %d" % (W, H, q, lam)}
    for i in range(a.warmup + a.iters):
        if i == a.warmup:
            w.prof_enable(True)
        w.TransformQuantize(img, W, 0, q, lam, on_device=True)
        w.prof_read()
    st = w.prof_read()
    out["wavelet_ms"] = {k: round(v[0] / v[1], 4) for k, v in st.items() if v[1]}
    fwd0 = out["wavelet_ms"].get("fwd_l0")
    if fwd0:
        out["fwd_l0_GBps"] = round(4.0 * W * H / (fwd0 * 1e-3) / 1e9, 1)
    enc = out["wavelet_ms"].get("fwd", 0) + out["wavelet_ms"].get("quant", 0)
    if enc:
        out["wavelet_encode_GBps"] = round(9.851 * W * H / (enc * 1e-3) / 1e9, 1)
    if a.codec:
        c = ric_amd.Codec(W, H, 1)
        dpix = torch.from_numpy(pix).cuda()
        dout = torch.empty_like(dpix)
        for i in range(a.warmup + a.iters):
            if i == a.warmup:
                c.prof_enable(True)
                t0 = time.perf_counter()
            ric = c.compress(dpix, q=9, trans=0, on_device=True)
            c.decompress(ric, pix_out=dout)
        dt = (time.perf_counter() - t0) / a.iters
        st = c.prof_read()
        out["codec_ms"] = {k: round(v[0] / v[1], 4) for k, v in st.items() if v[1]}
        out["codec_frame_ms"] = round(dt * 1e3, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
