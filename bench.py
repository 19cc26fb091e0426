#!/usr/bin/env python3
"""bench.py -- .ric encode+decode throughput on synthetic 8K grayscale frames.

Workload (BASELINE.json configs[2]): 7680x4320 8-bit gray,
5-level integer 9/7 wavelet, q=9, full .ric encode (DWT, RD quantiser,
zerotree + range coder) followed by the full decode (entropy decode,
dequantiser, inverse DWT, 8-bit output), bit-exact with the reference.

One step = every rank encodes and decodes its batch of frames.  Frames are
independent .ric streams, so ranks shard frames with no data-path collective
("scaling": "weak"); host worker threads run the serial range coder of
different frames concurrently while the GPU stages of all frames share the
device.  Inputs are resident in HBM before the timed region; outputs (decoded
frames) land in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--threads T]

Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rududu-image-codec_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0, help="frames per GPU per step (default: threads)")
    ap.add_argument("--threads", type=int, default=0, help="host coder threads per GPU (default 16)")
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--q", type=int, default=9)
    ap.add_argument("--trans", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=16)
    return ap.parse_args()


def cpu_baseline(w, h, q, trans, frames, threads):
    """Reference CPU path (oracle/_ref, the reference library compiled from its
    own sources; the clean-room port if absent), timed on this host's cores:
    `frames` independent 8K encode+decode round trips on `threads` threads."""
    sys.path.insert(0, REPO)
    from oracle import oracle as O
    chk = O.ref() or O.port()
    kind = "reference" if O.ref() is not None else "port"
    import ric_amd
    imgs = [ric_amd.synth(w, h, 1, 1000 + i) for i in range(frames)]

    def work(i):
        r = chk.encode_ric(imgs[i], q, trans)
        chk.decode_ric(r)

    t0 = time.perf_counter()
    ths = []
    for k in range(threads):
        def run(k=k):
            for i in range(k, frames, threads):
                work(i)
        ths.append(threading.Thread(target=run))
        ths[-1].start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    return {"value": round(frames * w * h / 1e6 / dt, 2), "unit": "Mpixel/s", "cores": threads, "kind": kind,
            "sample": "%d independent %dx%d gray q%d encode+decode round trips on %d host threads (%.1f s wall)"
                      % (frames, w, h, q, threads, dt)}


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import ric_amd
    W, H = a.width, a.height
    threads = a.threads or 16
    batch = a.batch or threads
    threads = min(threads, batch)

    # synthetic frames, uploaded to HBM before timing
    frames = []
    for i in range(batch):
        host = ric_amd.synth(W, H, 1, rank * batch + i)
        frames.append(torch.from_numpy(host).to(dev))
    outs = [torch.empty((1, H, W), dtype=torch.uint8, device=dev) for _ in range(batch)]
    torch.cuda.synchronize()

    codecs = [ric_amd.Codec(W, H, 1, device=local) for _ in range(threads)]
    sizes = [0] * batch
    errors = []

    def run_frames(k):
        c = codecs[k]
        try:
            for i in range(k, batch, threads):
                ric = c.compress(frames[i], q=a.q, trans=a.trans, on_device=True)
                sizes[i] = len(ric)
                c.decompress(ric, pix_out=outs[i])
        except Exception as e:  # surfaced after join
            errors.append(e)

    def step():
        ths = [threading.Thread(target=run_frames, args=(k,)) for k in range(threads)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errors:
            raise errors[0]

    for _ in range(a.warmup):
        step()
    for c in codecs:
        c.prof_enable(True)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt[0])

    # stage timers (HIP events on each codec's stream, summed over codecs)
    prof = {}
    for c in codecs:
        for k, (ms, n) in c.prof_read().items():
            s = prof.setdefault(k, [0.0, 0])
            s[0] += ms
            s[1] += n
    stage_ms = {k: round(v[0] / v[1], 4) for k, v in prof.items() if v[1]}

    # roofline of the dominant GPU kernel: the level-0 forward DWT
    # (algorithmic bytes, SURVEY.md §8(d): read the s16 plane + write 4 s16 bands = 4 B/px)
    fwd0_bytes = 4.0 * W * H
    t_fwd0 = stage_ms.get("fwd_l0")
    achieved = fwd0_bytes / (t_fwd0 * 1e-3) / 1e9 if t_fwd0 else None
    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_fwd_l0.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    # the whole GPU wavelet-encode stage (DWT + RD quantiser): 9.851 B/px at C3
    enc_gpu = (stage_ms.get("fwd", 0) + stage_ms.get("quant", 0)) or None

    total_px = world * batch * W * H * a.steps
    value = total_px / 1e6 / dt
    out = {
        "metric": "encode+decode Mpixel/s on 8K gray, 5-level wavelet; % HBM roofline",
        "value": round(value, 2),
        "unit": "Mpixel/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic (SURVEY.md §8(d) generator), resident in HBM",
        "config": {"workload": "C3: %dx%d gray, 5-level cdf97, q=%d, .ric encode+decode round trip, bit-exact"
                               % (W, H, a.q),
                   "frames_per_gpu_per_step": batch, "host_coder_threads_per_gpu": threads,
                   "parallelism": "frames sharded over %d GPU(s)" % world},
        "roofline": {"bound": "hbm", "kernel": "k_fwd (level 0 forward 9/7 DWT)",
                     "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "algorithmic_bytes_per_launch": fwd0_bytes,
                     "avg_launch_ms": t_fwd0},
        "gpu_wavelet_encode": {"ms": round(enc_gpu, 4) if enc_gpu else None,
                               "bytes": 9.851 * W * H,
                               "frac": round(9.851 * W * H / (enc_gpu * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                               if enc_gpu else None},
        "stage_ms": stage_ms,
        "bytes_per_frame": int(np.mean(sizes)),
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(W, H, a.q, a.trans, a.cpu_frames, min(16, a.cpu_frames))
        except Exception as e:
            out["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
