#!/usr/bin/env python3
"""gc_probe.py -- the GPU stream coder (ric_batch_encode_gpu) against the host
coder (ric_batch_encode) on the same frames: byte equality and time per
frame.  Development tool (GPU box).

    python scripts/gc_probe.py [--w 7680 --h 4320] [--n 16] [--q 9] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rududu-image-codec_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=7680)
    ap.add_argument("--h", type=int, default=4320)
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--q", type=int, default=9)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--check", type=int, default=4, help="frames compared with the host coder")
    a = ap.parse_args()
    import ric_amd
    frames = [ric_amd.DeviceArray.from_numpy(ric_amd.synth(a.w, a.h, 1, f)) for f in range(a.n)]
    b = ric_amd.Batch(a.w, a.h, 1, slots=a.n, threads=min(16, a.n))
    ostride = (a.w * a.h * 2 + 65536 + 4095) // 4096 * 4096
    out = ric_amd.DeviceArray(a.n * ostride, np.uint8, zero=True)
    t0 = time.time()
    lens = b.compress_gpu(frames, out, ostride, a.q, 0)
    ric_amd.device_sync()
    first = time.time() - t0
    best = 1e9
    for _ in range(a.reps):
        t0 = time.time()
        lens = b.compress_gpu(frames, out, ostride, a.q, 0)
        best = min(best, time.time() - t0)
    b.prof_enable(True)
    b.compress_gpu(frames, out, ostride, a.q, 0)
    p = b.prof_read()
    # the GPU stream decoder on the streams just written
    pix = [ric_amd.DeviceArray((1, a.h, a.w), np.uint8, zero=True) for _ in range(a.n)]
    b.decompress_gpu(out, ostride, lens, pix)
    ric_amd.device_sync()
    t0 = time.time()
    b.decompress_gpu(out, ostride, lens, pix)
    ric_amd.device_sync()
    dec_s = time.time() - t0
    b.prof_enable(True)
    b.decompress_gpu(out, ostride, lens, pix)
    pd = b.prof_read()
    host = out.numpy()
    nc = min(a.check, a.n)
    ref = b.compress([frames[i] for i in range(nc)], a.q, 0, on_device=True)
    ok = []
    for i in range(nc):
        g = host[i * ostride:i * ostride + lens[i]].tobytes()
        if g == ref[i]:
            ok.append(True)
            continue
        d = next((k for k in range(min(len(g), len(ref[i]))) if g[k] != ref[i][k]), min(len(g), len(ref[i])))
        print("frame %d: gpu %d bytes, host %d bytes, first difference at %d" % (i, len(g), len(ref[i]), d))
        ok.append(False)
    dok = []
    for i in range(nc):
        want = b.decompress([ref[i]])[0]
        dok.append(bool(np.array_equal(pix[i].numpy().reshape(want.shape), want)))
    t0 = time.time()
    nh = min(a.n, 16)                     # host coder reference timing on one group
    b.compress([frames[i] for i in range(nh)], a.q, 0, on_device=True)
    host_t = (time.time() - t0) * a.n / nh
    print(json.dumps({"w": a.w, "h": a.h, "n": a.n, "q": a.q, "equal": ok, "lens": lens[:4],
                      "gpu_encode_s": round(best, 4), "first_call_s": round(first, 3),
                      "gpu_frames_per_s": round(a.n / best, 2), "coder_kernel_ms": round(p["gpu_enc"][0], 2),
                      "host_encode_s_16thr": round(host_t, 4), "decode_equal": dok, "gpu_decode_s": round(dec_s, 4),
                      "decoder_kernel_ms": round(pd["gpu_dec"][0], 2)}))


if __name__ == "__main__":
    main()
