#!/usr/bin/env python3
"""bench.py -- .ric encode+decode throughput on synthetic 8K grayscale frames.

Workload (BASELINE.json configs[2]): 7680x4320 8-bit gray,
5-level integer 9/7 wavelet, q=9, full .ric encode (DWT, RD quantiser,
zerotree + range coder) followed by the full decode (entropy decode,
dequantiser, inverse DWT, 8-bit output), bit-exact with the reference.

One step = every rank encodes and decodes its batch of frames (default 64
per GPU, handed out dynamically to 16 host coder threads).  Frames are
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


def wavelet_bytes(W, H, levels=5, level_chg=1):
    """SURVEY.md §8(d) algorithmic byte model per level, at the reference's
    band types (s16 above level_chg, i32 at or below; ric: level_chg 1, so only
    the coarsest level is int):
      dwt[l]   read the level's input plane + write its 4 subbands;
      quant[l] read + write every coefficient of D, H, V + 8 B (pRD) per 4x4 block;
      deq[l]   read + write every coefficient of D, H, V (TSUQi);
      ll       the coarsest LL: TSUQ read + write (TSUQi the same, counted in deq)."""
    out = {"dwt": [], "quant": [], "deq": []}
    w, h = W, H
    in_sz = 2
    for l in range(levels):
        lv = levels - l              # the reference's level counter (wavelet2d.cpp:69-72)
        sz = 4 if lv <= level_chg else 2
        dD = ((w + 1) // 2) * ((h + 1) // 2)
        dV = ((w + 1) // 2) * (h // 2)
        dH = (w // 2) * ((h + 1) // 2)
        dL = (w // 2) * (h // 2)
        blk = sum(((bx + 3) // 4) * ((by + 3) // 4) for bx, by in
                  (((w + 1) // 2, (h + 1) // 2), ((w + 1) // 2, h // 2), (w // 2, (h + 1) // 2)))
        coef = dD + dV + dH
        out["dwt"].append(w * h * in_sz + (coef + dL) * sz)
        out["quant"].append(coef * 2 * sz + 8 * blk)
        out["deq"].append(coef * 2 * sz)
        w, h, in_sz = w // 2, h // 2, sz
        last_sz = sz
    out["ll"] = w * h * 2 * last_sz
    out["deq"][-1] += out["ll"]
    return out


def _frac(ms, nbytes):
    if not ms:
        return {"ms": None, "bytes": nbytes, "frac": None}
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {"ms": round(ms, 4), "bytes": nbytes, "GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0, help="frames per GPU per step (default: 8 per host thread)")
    ap.add_argument("--threads", type=int, default=0, help="host coder threads per GPU (default 16)")
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--q", type=int, default=9)
    ap.add_argument("--trans", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the per-step stream gather to rank 0")
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
    # one process per GPU; a rehearsal with more ranks than GPUs (gloo) wraps
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # one process per GPU; barrier, max-over-ranks timing and the final stream
    # gather go over RCCL ("nccl" is RCCL on ROCm; RIC_BENCH_BACKEND=gloo for a
    # CPU-side rehearsal)
    backend = os.environ.get("RIC_BENCH_BACKEND", "nccl")
    cdev = dev if backend == "nccl" else torch.device("cpu")
    if world > 1:
        dist.init_process_group(backend, init_method="env://")

    def barrier():
        if world > 1:
            t = torch.ones(1, device=cdev)
            dist.all_reduce(t)

    import ric_amd
    import shard
    W, H = a.width, a.height
    threads = a.threads or 16
    # 8 frames per host coder thread: the threads drift apart after their
    # first frame, so their exclusive GPU sections stop queueing behind one
    # another, and the idle tail at the end of a step (threads waiting for the
    # last frames) shrinks with the frames per thread (one box, 16 threads:
    # 16 frames per step 1490-1750 Mpix/s, 64: 2023, 128: 2072, 256: 2089)
    batch = a.batch or 8 * threads
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

    # frames are handed out dynamically (next free frame), so the host coder
    # threads drift apart after their first frame and their exclusive GPU
    # sections interleave with the other threads' host work
    next_frame = [0]
    lock = threading.Lock()

    def run_frames(k):
        c = codecs[k]
        try:
            while True:
                with lock:
                    i = next_frame[0]
                    next_frame[0] += 1
                if i >= batch:
                    break
                ric = c.compress(frames[i], q=a.q, trans=a.trans, on_device=True)
                sizes[i] = len(ric)
                streams[i] = ric
                c.decompress(ric, pix_out=outs[i])
        except Exception as e:  # surfaced after join
            errors.append(e)

    gather = world > 1 and not a.no_gather
    streams = [b""] * batch
    gathered = [0]

    def step():
        next_frame[0] = 0
        ths = [threading.Thread(target=run_frames, args=(k,)) for k in range(threads)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errors:
            raise errors[0]
        if gather:
            # the path's one exchange: every rank's .ric streams to rank 0
            # (SURVEY.md §8(e)); rank 0 keeps them on the device
            got = shard.gather_streams(streams, dist, device=cdev, to_host=False)
            if rank == 0:
                gathered[0] = int(sum(int(s[1:1 + int(s[0])].sum()) for s in got[1]))

    for _ in range(a.warmup):
        step()
    for c in codecs:
        c.prof_enable(True)

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    barrier()
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=cdev)
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

    # roofline of the dominant GPU kernel: the level-0 launch of the fused
    # forward 9/7 DWT + RD quantiser + zerotree records (dwt.hip k_fwdq_pc).
    # Algorithmic bytes = SURVEY.md §8(d)'s per-unit figures for the work that
    # one launch does: the level-0 DWT (4 B/px) plus the level-0 quantiser
    # (read + write every s16 coefficient, 4 B/coef, + 8 B per 4x4 block).
    bm = wavelet_bytes(W, H)
    l0_bytes = bm["dwt"][0] + bm["quant"][0]
    t_fwd0 = stage_ms.get("fwd_l0")
    achieved = l0_bytes / (t_fwd0 * 1e-3) / 1e9 if t_fwd0 else None
    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_fwd_l0.json")
    if os.path.exists(pmc):
        try:
            p = json.load(open(pmc))
            if p.get("kernel", "").startswith("k_fwdq_pc"):
                traffic = p.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    # the whole GPU wavelet encode (every forward level + quantiser + LL TSUQ):
    # the §8(d) DWT + quant model, 326.8 MB at C3
    enc_bytes = sum(bm["dwt"]) + sum(bm["quant"]) + bm["ll"]
    enc_gpu = (stage_ms.get("fwd", 0) + stage_ms.get("quant", 0)) or None
    # the GPU decode stages: dequantiser (r + w) + inverse DWT (= forward bytes)
    dec_bytes = sum(bm["dwt"]) + sum(bm["deq"])
    dec_gpu = (stage_ms.get("dequant", 0) + stage_ms.get("inv", 0)) or None

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
        "roofline": {"bound": "hbm",
                     "kernel": "k_fwdq_pc level 0 (fused forward 9/7 DWT + RD quantiser + block records)",
                     "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "algorithmic_bytes_per_launch": l0_bytes,
                     "avg_launch_ms": t_fwd0},
        "gpu_wavelet_encode": _frac(enc_gpu, enc_bytes),
        "gpu_wavelet_decode": _frac(dec_gpu, dec_bytes),
        "stage_ms": stage_ms,
        "bytes_per_frame": int(np.mean(sizes)),
    }
    if gather:
        out["gather"] = {"backend": backend, "bytes_to_rank0_per_step": gathered[0]}
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
