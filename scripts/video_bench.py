#!/usr/bin/env python3
"""video_bench.py -- the video codec (ric_video: CRududuCodec on the GPU) on a
synthetic panning sequence: end-to-end encode and decode frames/s, and, with
--kstats <rocprofv3 kernel_stats.csv>, each motion kernel's time per frame and
its fraction of the HBM roofline from the algorithmic byte model below.

    python scripts/video_bench.py [--w 1920 --h 1080 --frames 30 --q 20]
    rocprofv3 --kernel-trace --stats -d gpurun_out/vk -o run -- python3 scripts/video_bench.py ...
    python scripts/video_bench.py --kstats gpurun_out/vk/.../run_kernel_stats.csv --w 1920 --h 1080 --frames 30

Algorithmic bytes per frame (int16 samples, 3 planes of w x h, P = 3 w h):
  k_vid_interp     read sub[0] once + write the 15 other quarter-pel images: 32 B x P
  k_vid_extend     16 images x 3 planes x the border ring (15 samples deep):
                   read + write 2 B each
  k_vid_obmc       per predicted sample: the old prediction read + written and
                   the 4 overlapping blocks' source samples: 12 B x 3 x 8bx x 8by;
                   the encoder's launches also take the residual (image read +
                   written, 4 B x P), the decoder's do not: the average over
                   the equal numbers of both is 12 B x 3 x 64 bx by + 2 B x P
  k_vid_addsub     read two images, write one: 6 B x P (once per encoded and
                   once per decoded inter frame: the reconstruction)
  k_vid_input      3 B in, 6 B out per pixel
  k_vid_epzs_sub   per block: the current block + 16 candidate blocks, 128 B each
  k_vid_epzs_full  latency-bound wavefront (one wave per block row; a block
                   waits for the row above): reported as time, not as bandwidth
HBM peak 8.0 TB/s (MI355X_MICROARCH.md)."""
import argparse
import csv
import json
import os
import re
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rududu-image-codec_amd"), os.path.join(REPO, "tests")]
PEAK = 8000.0


def model(w, h):
    P = 3 * w * h
    bx, by = w >> 3, h >> 3
    ring = 2 * 15 * (w + 30) + 30 * h
    return {"k_vid_interp": 32 * P, "k_vid_extend": 16 * 3 * ring * 4, "k_vid_obmc": 12 * 3 * 64 * bx * by + 2 * P,
            "k_vid_addsub": 6 * P, "k_vid_input": 9 * w * h, "k_vid_epzs_sub": 17 * 128 * bx * by}


def kstats(path, w, h, frames, inter):
    m = model(w, h)
    out = {}
    for row in csv.DictReader(open(path)):
        name = row.get("Name") or row.get("KernelName") or ""
        mk = re.search(r"k_vid_\w+", name)
        if not mk:
            continue
        short = mk.group(0)
        calls = int(row["Calls"])
        avg_ns = float(row["AverageNs"])
        rec = {"calls": calls, "avg_us": round(avg_ns / 1e3, 2), "total_ms": round(calls * avg_ns / 1e6, 3)}
        if short in m and short != "k_vid_addsub":
            gbs = m[short] / (avg_ns * 1e-9) / 1e9
            rec.update({"bytes_per_launch": m[short], "GBps": round(gbs, 1), "hbm_frac": round(gbs / PEAK, 4)})
        elif short == "k_vid_addsub":
            gbs = m[short] / (avg_ns * 1e-9) / 1e9
            rec.update({"bytes_per_launch": m[short], "GBps": round(gbs, 1), "hbm_frac": round(gbs / PEAK, 4)})
        out[short] = rec
    return out


def pmc(fetch_csv, write_csv):
    """HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE passes (KiB per
    dispatch; MI355X_MICROARCH.md: on gfx950 FETCH_SIZE counts half the bytes
    of a wide coalesced read, so the read side is doubled; the raw value is
    kept; Infinity-Cache hits are counted, not excluded)."""
    acc = {}
    for path, key in ((fetch_csv, "FETCH_SIZE"), (write_csv, "WRITE_SIZE")):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") != key:
                continue
            mk = re.search(r"k_vid_\w+", r["Kernel_Name"])
            if not mk:
                continue
            short = mk.group(0)
            acc.setdefault(short, {}).setdefault(key, []).append(float(r["Counter_Value"]) * 1024)
    out = {}
    for k, d in acc.items():
        f = float(np.mean(d.get("FETCH_SIZE", [0])))
        w = float(np.mean(d.get("WRITE_SIZE", [0])))
        out[k] = {"traffic_bytes": int(2 * f + w), "fetch_raw_bytes": int(f), "write_bytes": int(w)}
    return out


def cpu_baseline(seq, q):
    """the reference video codec (oracle/_ref/ricvid_ref: its classes compiled
    from the reference sources, -O2, single-threaded as the reference is) on
    the first frames of the same sequence, encode and decode timed apart"""
    import subprocess
    import tempfile
    import video_seq
    if not os.path.exists(video_seq.REF_BIN):
        return None
    n, _, h, w = seq.shape
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "seq.rgb")
        np.ascontiguousarray(seq).tofile(src)
        r = subprocess.run([video_seq.REF_BIN, str(w), str(h), str(q), str(n), src, "/dev/null"],
                           env=dict(os.environ, RICVID_TIME="1"), capture_output=True, text=True, timeout=600, check=True)
    t = json.loads(r.stderr.strip().splitlines()[-1])
    return {"kind": "reference", "cores": 1, "frames": n, "encode_fps": round(n / t["encode_s"], 3),
            "decode_fps": round(n / t["decode_s"], 3), "sample": "the first %d frames of the same sequence" % n}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--q", type=int, default=20)
    ap.add_argument("--host-threads", type=int, default=8, help="the encoder's serial stage (ric_video_set_host_threads)")
    ap.add_argument("--cpu-frames", type=int, default=10,
                    help="frames of the same sequence through oracle/_ref/ricvid_ref (0: skip)")
    ap.add_argument("--kstats", default=None)
    ap.add_argument("--pmc", nargs=2, default=None, metavar=("FETCH_CSV", "WRITE_CSV"),
                    help="counter_collection.csv of the FETCH_SIZE and WRITE_SIZE passes")
    a = ap.parse_args()
    inter = a.frames - (a.frames + 9) // 10
    if a.kstats:
        ks = kstats(a.kstats, a.w, a.h, a.frames, inter)
        if a.pmc:
            for k, t in pmc(a.pmc[0], a.pmc[1]).items():
                if k in ks:
                    ks[k].update(t)
        print(json.dumps({"w": a.w, "h": a.h, "frames": a.frames, "kernels": ks}))
        return
    import ric_amd
    import video_seq
    seq = video_seq.sequence(a.w, a.h, a.frames, 1)
    dev = [ric_amd.DeviceArray.from_numpy(np.ascontiguousarray(f)) for f in seq]
    enc = ric_amd.VideoCodec(True, a.w, a.h)
    dec = ric_amd.VideoCodec(False, a.w, a.h)
    enc.quant = dec.quant = a.q
    enc.set_host_threads(a.host_threads)
    # warm up on a separate pair (the codec's state is the sequence's)
    we, wd = ric_amd.VideoCodec(True, a.w, a.h), ric_amd.VideoCodec(False, a.w, a.h)
    we.quant = wd.quant = a.q
    for k in range(3):
        wd.decode(we.encode(dev[k]))
    del we, wd
    streams = []
    t0 = time.perf_counter()
    for f in dev:
        streams.append(enc.encode(f))
    te = time.perf_counter() - t0
    t0 = time.perf_counter()
    for s in streams:
        dec.decode(s)
    td = time.perf_counter() - t0
    mpx = a.w * a.h / 1e6
    cpu = cpu_baseline(seq[:a.cpu_frames], a.q) if a.cpu_frames > 0 else None
    print(json.dumps({"cpu_baseline": cpu, "host_threads": a.host_threads,"workload": "video: CRududuCodec %dx%d RGB, quant %d, %d frames (key every 10)"
                                  % (a.w, a.h, a.q, a.frames),
                      "encode_fps": round(a.frames / te, 2), "decode_fps": round(a.frames / td, 2),
                      "encode_ms_per_frame": round(te / a.frames * 1e3, 2), "decode_ms_per_frame": round(td / a.frames * 1e3, 2),
                      "encode_mpix_s": round(a.frames * mpx / te, 1), "decode_mpix_s": round(a.frames * mpx / td, 1),
                      "bytes_per_frame": int(np.mean([len(s) for s in streams]))}))


if __name__ == "__main__":
    main()
