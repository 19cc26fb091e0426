#!/usr/bin/env python3
"""bench.py -- .ric encode+decode throughput on synthetic frames (MI355X).

Workloads (BASELINE.json configs):
  C3 (default)  7680x4320 8-bit gray, 5-level integer 9/7, q=9: full .ric
                encode (DWT, RD quantiser, zerotree records, range coder)
                followed by the full decode (entropy decode, fused TSUQi +
                inverse DWT, 8-bit output), bit-exact with the reference.
                Each rank codes its own frames (weak scaling).
  C5            64 independent 4096x4096 gray frames per step in total,
                frame f on rank f mod N (strong scaling).
  C4            one 7680x4320 RGB image as 2x2 tiles of 3840x2160, tile
                (tx, ty) on rank 2*ty + tx (round robin when N < 4), the four
                tile streams gathered to rank 0 into an RTL1 container.

One step = every rank encodes and decodes its frames through ric_batch: the
frames of a group (`--slots`, default one per host thread) go through every
GPU level as one launch (blockIdx.z = frame), a native pool of host coder
threads runs the serial range coder of different frames, and the GPU stages
of one group overlap the host coding of the previous one.  Inputs are
resident in HBM before the timed region; decoded frames land in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C3|C4|C5]
                    [--frames F] [--threads T] [--slots S]

Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
(one process per GPU; barrier and max-over-ranks timing over gloo on the CPU;
the stream gather to rank 0 over the library's RCCL communicator, overlapped
with the step).  Device memory comes from the library itself
(ric_amd.DeviceArray): torch is imported only for torch.distributed's CPU
process group, and never touches the GPU.
"""
import argparse
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rududu-image-codec_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)
# a reference C3 (8K gray q9) encode makes 19.24 M
# codeBin and 19.26 M bitsCode calls -- the serial stage's event count
C3_EVENTS = 19.24e6 + 19.26e6


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
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="C3", choices=["C3", "C4", "C5"])
    ap.add_argument("--frames", type=int, default=0,
                    help="C3: frames per GPU per step (default 8 per host thread); C5: frames per step in total (64)")
    ap.add_argument("--batch", type=int, default=0, help="alias of --frames")
    ap.add_argument("--threads", type=int, default=0, help="host coder threads per GPU (default: this rank's CPU share)")
    ap.add_argument("--slots", type=int, default=0, help="frames per GPU launch group (default: --threads)")
    ap.add_argument("--q", type=int, default=9)
    ap.add_argument("--trans", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-latency", action="store_true", help="skip the one-frame ric_codec latency after timing")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the per-step stream gather to rank 0")
    ap.add_argument("--no-split", action="store_true", help="skip the encode-only / decode-only timing")
    ap.add_argument("--coder", default=None, choices=["host", "hybrid", "gpu", "mix"],
                    help="serial coder: host threads; hybrid = GPU stream encoder + host decoder; gpu = GPU stream "
                         "encoder and decoder (one wave per stream), host threads doing whole round trips beside it; "
                         "mix = GPU stream encoder, each launch decoded by the host threads or the GPU stream decoder "
                         "(whichever has room)")
    ap.add_argument("--pool", type=int, default=1536,
                    help="hybrid / gpu: frames per GPU stream-coder launch (two in flight: 3072 = three coder waves "
                         "on every SIMD; shrunk to fit memory)")
    ap.add_argument("--value-cap", type=int, default=-1,
                    help="hybrid / gpu: the pool's compacted level-0 value capacity per frame plane "
                         "(ric_batch_hybrid_config_ex: -1 the default 9/16 of the coefficients, 0 dense bands)")
    ap.add_argument("--launches", type=int, default=2, help="hybrid / gpu: stream-coder launches per step")
    ap.add_argument("--distinct", type=int, default=128,
                    help="distinct frames resident in HBM (inputs, outputs) and host stream buffers; a longer step cycles them")
    ap.add_argument("--n-host", type=int, default=-1,
                    help="hybrid / gpu / mix: frames per step round-tripped by the host threads beside the GPU stream "
                         "coder (default: gpu 50 per thread, else 16 per thread)")
    a = ap.parse_args()
    if a.coder is None:   # C3 (one large gray frame per stream): the GPU stream coder; C4 (RGB) / C5: host
        a.coder = "gpu" if a.workload == "C3" else "host"
    return a


def default_n_host(a, threads):
    return a.n_host if a.n_host >= 0 else (50 if a.coder == "gpu" else 16) * threads


def host_frames_room(a, threads):
    """Host round trips a step has frames for: with --coder gpu and no --n-host
    the split is balanced after the warmup (up to 112 per thread)."""
    return 112 * threads if (a.n_host < 0 and a.coder == "gpu") else default_n_host(a, threads)


def host_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    quota = None
    try:                                   # cgroup v2 CPU quota ("max" = none)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota, "model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def default_threads(world):
    """This rank's share of the host: OMP_NUM_THREADS when the launcher sets
    it (16 per GPU on the GPU boxes), else the affinity mask split over the
    ranks of the node."""
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        return int(omp)
    hi = host_info()
    return max(1, min(32, (hi["affinity_cpus"] or 1) // max(world, 1)))


def cpu_baseline(W, H, q, trans, threads, per_thread=2):
    """The reference CPU path (oracle/_ref: the reference library compiled
    from its own sources; the clean-room port if absent), on this host:
    (i) one stream on one core (latency), (ii) independent streams on
    `threads` threads (this GPU's CPU share) and on the node's per-GPU share
    of its cores (nproc / 8) when that is larger (throughput); encode and
    decode timed separately, `per_thread` frames per thread.  `value` is the
    best throughput point, `cores` its thread count."""
    sys.path.insert(0, REPO)
    from oracle import oracle as O
    chk = O.ref() or O.port()
    kind = "reference" if O.ref() is not None else "port"
    import ric_amd
    chk.decode_ric(chk.encode_ric(ric_amd.synth(64, 48, 1, 0), q, trans))   # lazy statics (init_lut) first
    mpx = W * H / 1e6

    def run(nthreads, per):
        imgs = [[ric_amd.synth(W, H, 1, 1000 + k * per + i) for i in range(per)] for k in range(nthreads)]
        rics = [[None] * per for _ in range(nthreads)]

        def enc(k):
            for i in range(per):
                rics[k][i] = chk.encode_ric(imgs[k][i], q, trans)

        def dec(k):
            for i in range(per):
                chk.decode_ric(rics[k][i])

        out = {}
        for name, fn in (("encode", enc), ("decode", dec)):
            ths = [threading.Thread(target=fn, args=(k,)) for k in range(nthreads)]
            t0 = time.perf_counter()
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            out[name] = time.perf_counter() - t0
        n = nthreads * per
        return {"threads": nthreads, "frames": n, "encode_mpix_s": round(n * mpx / out["encode"], 2),
                "decode_mpix_s": round(n * mpx / out["decode"], 2),
                "roundtrip_mpix_s": round(n * mpx / (out["encode"] + out["decode"]), 2),
                "wall_s": round(out["encode"] + out["decode"], 2)}

    hi = host_info()
    lat = run(1, 1)
    points = [run(threads, per_thread)]
    node_share = (hi["nproc"] or 0) // 8
    quota = hi["cgroup_cpu_quota"]
    # the CPUs this process is actually granted: the affinity mask and the
    # cgroup quota (more threads than that only time-share the same CPUs)
    granted = min(x for x in (hi["affinity_cpus"] or node_share or threads, int(quota) if quota else None, 1 << 30)
                  if x)
    if node_share > threads and granted > threads:
        points.append(run(min(node_share, granted), 1))
    best = max(points, key=lambda p: p["roundtrip_mpix_s"])
    return {"value": best["roundtrip_mpix_s"], "unit": "Mpixel/s", "cores": min(best["threads"], granted), "kind": kind,
            "sample": "%dx%d gray q%d frames, encode then decode: 1 frame on 1 thread (latency); %s (throughput); "
                      "value = the best throughput point (%d threads)"
                      % (W, H, q, ", ".join("%d frames on %d threads (%.1f s)" % (p["frames"], p["threads"], p["wall_s"])
                                            for p in points), best["threads"]),
            "headline_cores": "%d threads on %d granted CPUs: %s%s" % (best["threads"], min(best["threads"], granted), "this GPU's CPU share (OMP_NUM_THREADS)"
                                                    if best["threads"] == threads else
                                                    "the node's per-GPU share of its cores (nproc / 8)",
                                                    "; the process's cgroup CPU quota is %s CPUs" % hi["cgroup_cpu_quota"]
                                                    if hi["cgroup_cpu_quota"] else ""),
            "latency_1core": lat, "throughput_points": points, "host": hi}


def pixel_digest(pix):
    """ric_batch_set_digests' digest (include/ric_gpu.h) of one decoded frame:
    sum over byte k of pix[k] * (k * 0x9E3779B97F4A7C15 + 1), mod 2^64."""
    flat = np.ascontiguousarray(pix, np.uint8).reshape(-1).astype(np.uint64)
    mult = np.arange(flat.size, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1)
    return np.uint64(np.sum(flat * mult, dtype=np.uint64))


def oracle_expectations(host_frames, q, trans, threads):
    """The reference CPU path (oracle/_ref: the reference library compiled from
    its own sources; the clean-room port when absent) on each input, on a pool
    of `threads` threads: [(.ric bytes, decoded planes)], wall seconds, kind.
    Checker only: used after the timed region."""
    sys.path.insert(0, REPO)
    from oracle import oracle as O
    from concurrent.futures import ThreadPoolExecutor
    chk = O.ref() or O.port()
    kind = "reference" if O.ref() is not None else "port"
    h, w = host_frames[0].shape[-2:]
    import ric_amd
    chk.decode_ric(chk.encode_ric(ric_amd.synth(64, 48, host_frames[0].shape[0], 0), q, trans))   # lazy statics first

    def one(img):
        r = chk.encode_ric(img, q, trans)
        return r, chk.decode_ric(r)[0].reshape(img.shape)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max(1, threads)) as ex:
        res = list(ex.map(one, host_frames))
    return res, time.perf_counter() - t0, kind


def workload_frames(a, rank, world, threads):
    """(W, H, channels, [(global index, synth frame, crop)], scaling)"""
    if a.workload == "C3":
        W, H = 7680, 4320
        if getattr(a, "coder", "host") in ("hybrid", "gpu", "mix"):
            # two stream-coder launches in flight plus the host threads' round trips
            n = a.frames or a.batch or getattr(a, "launches", 2) * a.pool + host_frames_room(a, threads)
        else:
            n = a.frames or a.batch or 8 * threads
        return W, H, 1, [(rank * n + i, rank * n + i, None) for i in range(n)], "weak"
    if a.workload == "C5":
        W, H = 4096, 4096
        total = a.frames or a.batch or 64
        import shard
        return W, H, 1, [(f, f, None) for f in shard.frames_of_rank(total, world, rank)], "strong"
    import shard
    rects = shard.tile_rects(7680, 4320)
    mine = [(i, 0, rects[i]) for i in shard.tiles_of_rank(world, rank)]
    return 3840, 2160, 3, mine, "strong"


def main():
    t_start = time.perf_counter()
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the library (and its HIP runtime) first; torch only for the CPU process group
    import ric_amd
    import shard
    ndev = ric_amd.lib().ric_device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no HIP device visible")
    # one process per GPU; a rehearsal with more ranks than GPUs (gloo) wraps
    local = local % ndev
    # the gather's transport: RCCL (the library's communicator, xGMI) or, for a
    # rehearsal with several ranks on one GPU, gloo on the CPU
    backend = os.environ.get("RIC_BENCH_BACKEND", "rccl")
    dist = None
    transport = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")
        if backend == "gloo":
            transport = shard.GlooTransport(dist)
        else:
            backend = "rccl"
            uid = [ric_amd.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            transport = shard.RcclTransport(ric_amd.Comm(uid[0], world, rank, local), local)

    def barrier():
        if world > 1:
            dist.barrier()

    def allreduce(v, op):
        if world == 1:
            return v
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op])
        return float(t[0])

    def dsync():
        ric_amd.device_sync(local)

    threads = a.threads or default_threads(world)
    W, H, CH, mine, scaling = workload_frames(a, rank, world, threads)
    nfr = len(mine)
    slots = max(1, min(a.slots or threads, max(nfr, 1)))

    # synthetic frames, uploaded to HBM before timing
    # at most --distinct distinct frames in HBM (inputs and outputs): a longer
    # step reuses them cyclically; every frame is still encoded and decoded in full
    frames, rgb = [], None
    for k, (_, f, crop) in enumerate(mine):
        if k and k % 32 == 0 and k < a.distinct and rank == 0:
            print("[bench] frames %d/%d" % (k, min(nfr, a.distinct)), file=sys.stderr, flush=True)
        if k >= a.distinct:
            frames.append(frames[k % a.distinct])
            continue
        if crop is None:
            host = ric_amd.synth(W, H, CH, f)
        else:
            if rgb is None:
                rgb = ric_amd.synth(7680, 4320, 3, 0)
            _, _, x0, y0, w, h = crop
            host = np.ascontiguousarray(rgb[:, y0:y0 + h, x0:x0 + w])
        frames.append(ric_amd.DeviceArray.from_numpy(host, local))
    # decoded-frame buffers cycled over the distinct inputs (frames k and
    # k + distinct decode the same input); every frame's output is checked
    # after the timed region through its digest, taken by the library in
    # stream order right after the frame's pixels are written
    # (ric_batch_set_digests), so a later frame reusing the buffer hides
    # nothing.  (One buffer per frame would take ~100 GB of HBM at C3, which
    # the stream coder's pool uses instead.)
    nout = min(nfr, a.distinct)
    outs_d = [ric_amd.DeviceArray((CH, H, W), np.uint8, local) for _ in range(nout)]
    outs = [outs_d[k % nout] for k in range(nfr)]
    digests = ric_amd.DeviceArray(max(nfr, 1), np.uint64, local, zero=True)
    dsync()

    b = ric_amd.Batch(W, H, CH, slots=slots, threads=threads, device=local) if nfr else None
    if b is not None:
        b.set_digests(digests, nfr)
    gather = world > 1 and not a.no_gather
    gathered = [0]
    container = [None]
    # the path's one exchange: every stream this rank codes
    # goes to rank 0 in bounded chunks while the step runs (shard.StreamGather):
    # a stream leaves as soon as its .ric file is complete (ric_batch_set_ready)
    ready = np.zeros(max(nfr, 1), np.uint32)
    gath = None
    gstats = {"rounds": 0, "streams": 0, "bytes": 0, "digest_mismatches": 0, "tail_ms": []}
    if gather and a.workload != "C4":
        # allocated before the stream coder's pool, which takes the rest of HBM
        gath = shard.StreamGather(transport, rank, world, chunk_bytes=64 << 20)
        if b is not None:
            b.set_ready(ready, nfr)

    hybrid = a.coder in ("hybrid", "gpu", "mix") and b is not None
    gpu_dec = {"hybrid": 0, "gpu": 1, "mix": 2}.get(a.coder, 0)
    n_host = 0
    nstep = nfr                                # frames coded per step
    if hybrid:
        n_host = min(nfr, default_n_host(a, threads))
        # the stream coder's frames: two launches in flight (or the rest of --frames)
        n_gpu = nfr - n_host if (a.frames or a.batch) else min(a.launches * a.pool, nfr - n_host)
        nstep = n_host + n_gpu
        # stream capacity: 3 bits per pixel (a q9 C3 stream is 1.7; lossless q0
        # up to 10), 16-byte multiple
        pool = min(a.pool, max(n_gpu, 1))
        scap = (W * H * CH * (10 if a.q == 0 else 3) // 8 + 65536) // 16 * 16
        # the pool holds bands (the finest level compacted) + records + a
        # stream per frame in flight (C3: ~79 MB; 98 MB with dense bands): if
        # it does not fit this GPU's memory, shrink it
        while True:
            try:
                b.hybrid_config(pool, scap, a.value_cap)
                break
            except ric_amd.RicError as e:
                if e.rc != ric_amd.RIC_E_CAPACITY or pool <= 64:
                    raise
                print("[bench] a stream coder pool of %d frames does not fit: %d" % (pool, pool - 64),
                      file=sys.stderr, flush=True)
                pool -= 64
        b.cp_pool = pool
        if not (a.frames or a.batch):
            n_gpu = min(a.launches * pool, nfr - n_host)
            nstep = n_host + n_gpu
        # one host buffer per frame's .ric file (the library rejects aliased
        # buffers: host coders and the stream copier write them concurrently)
        sbufs = [np.empty(scap, np.uint8) for _ in range(nfr)]

    def host_stream(i, ln):
        return (sbufs[i] if hybrid else b._outs[i])[:ln]

    def step():
        th, gres, failed = None, {}, [False]
        if gath is not None:
            ready[:] = 0
            m = (n_host + n_gpu) if hybrid else nfr

            def stop():
                if failed[0]:
                    raise RuntimeError("the step failed")

            def run():
                try:
                    if rank == 0:
                        gres.update(gath.receive())
                    else:
                        gres.update(gath.send(m if b is not None else 0, ready, host_stream, stop=stop))
                    gres["t_end"] = time.perf_counter()
                except Exception as e:           # reported by the main thread
                    gres["error"] = repr(e)
            th = threading.Thread(target=run)
            th.start()
        try:
            if b is not None:
                if hybrid:
                    m = n_host + n_gpu
                    b.roundtrip_hybrid(frames[:m], outs[:m], n_host, q=a.q, trans=a.trans, gpu_decode=gpu_dec,
                                       streams=sbufs[:m])
                else:
                    b.roundtrip(frames, outs, q=a.q, trans=a.trans)
        except Exception:
            failed[0] = True
            raise
        t_coded = time.perf_counter()
        if th is not None:
            th.join()
            if "error" in gres:
                raise RuntimeError("rank %d: stream gather failed: %s" % (rank, gres["error"]))
            gstats["rounds"] += gres["rounds"]
            gstats["tail_ms"].append(round((gres["t_end"] - t_coded) * 1e3, 1))
            if rank == 0:
                gstats["streams"] += sum(gres["streams"]) + (n_host + n_gpu if hybrid else nfr)
                gstats["bytes"] += sum(gres["bytes"]) + (sum(b._lens) if b is not None else 0)
                gstats["digest_mismatches"] += len(gres["digest_mismatches"])
                gathered[0] = gstats["bytes"]
        if gather and a.workload == "C4":
            # C4: the tile streams to rank 0 into one RTL1 container, and the
            # decode side of the exchange: the container's tiles scattered
            # back to the ranks that decode them (shard.scatter_streams)
            streams = [b.stream(i) for i in range(nfr)] if b is not None else []
            got = shard.gather_streams(streams, transport, rank, world)
            per_rank = None
            if rank == 0:
                tiles = [None] * 4
                for r, lst in enumerate(got):
                    for i, s in zip(shard.tiles_of_rank(world, r), lst):
                        tiles[i] = s
                container[0] = shard.pack_tiles(7680, 4320, 2, 2, tiles)
                gathered[0] = len(container[0])
                _, _, _, _, back = shard.unpack_tiles(container[0])
                per_rank = [[back[i] for i in shard.tiles_of_rank(world, r)] for r in range(world)]
            mine_back = shard.scatter_streams(per_rank, transport, rank, world)
            if mine_back != streams:
                raise RuntimeError("rank %d: scattered tile streams differ from the encoded ones" % rank)

    def progress(what):
        # a line on stderr per step: a step with the stream coder takes seconds
        # and the harness takes a silent run for a hung one
        if rank == 0:
            print("[bench] %s %.1f s" % (what, time.perf_counter() - t_start), file=sys.stderr, flush=True)

    # Host/GPU split (--coder gpu, no --n-host): the last warmup step measures a
    # host round trip per thread and a stream-coder launch pair (encode +
    # decode: the GPU side of a step), and the host threads then take as many
    # round trips as fit in the GPU side's time, so neither side idles.
    balance = None
    auto = hybrid and gpu_dec == 1 and a.n_host < 0 and not (a.frames or a.batch) and a.warmup >= 2
    t_warm = None
    for i in range(a.warmup):
        if auto and i == a.warmup - 1:
            b.prof_enable(True)
            t_warm = time.perf_counter()
        step()
        if t_warm is not None and i == a.warmup - 1:
            t_warm = (time.perf_counter() - t_warm) * 1e3
        progress("warmup step %d/%d" % (i + 1, a.warmup))
    if auto:
        pw = b.prof_read()
        per_warm = n_host // threads
        per, t_host, t_gpu, t_eff, th, tg = per_warm, 0.0, 0.0, 0.0, 0.0, 0.0
        coded = (pw["gpu_enc"][2] and pw["gpu_dec"][2]) or pw["gpu_rt"][2]
        if pw["host_enc"][1] and coded:
            t_host = (pw["host_enc"][0] + pw["host_dec"][0]) / pw["host_enc"][1]     # ms per round trip per thread
            if pw["gpu_rt"][2]:                    # encode + decode as one kernel (k_gc_roundtrip)
                t_gpu = pw["gpu_rt"][0] / pw["gpu_rt"][2]
            else:
                t_gpu = pw["gpu_enc"][0] / pw["gpu_enc"][2] + pw["gpu_dec"][0] / pw["gpu_dec"][2]
            # the warmup step's own timeline: when the host side (its last round
            # trip group) and the GPU side (its last coder batch) finished; the
            # host share is scaled so both end together (a little before the GPU)
            th, tg = b.hybrid_times()
            # host round trips per step, not a whole number per thread: the host
            # pool takes them in groups, so a step may give some threads one more
            if th > 0 and tg > 0:
                t_eff = th / per_warm                       # host wall ms per round trip per thread
                nh = int(threads * per_warm * (tg - 150.0) / th)
            else:
                t_eff = 1.08 * t_host
                nh = int(threads * t_gpu / t_eff)
            per = max(threads, min(nh, host_frames_room(a, threads))) / threads
        per = allreduce(per, "min")           # one split for every rank: the slowest rank's
        n_host = min(int(round(per * threads)), nfr - n_gpu)
        nstep = n_host + n_gpu
        balance = {"host_round_trip_ms": round(t_host, 1), "host_wall_ms_per_frame": round(t_eff, 1),
                   "gpu_launch_pair_ms": round(t_gpu, 1), "warmup_step_ms": round(t_warm, 1),
                   "warmup_host_side_ms": round(th, 1), "warmup_gpu_side_ms": round(tg, 1),
                   "host_frames_per_thread": round(per, 2)}
        progress("balance: host side %.0f ms, GPU side %.0f ms in the last warmup step -> %.2f host frames per thread"
                 % (th, tg, per))
    if b is not None:
        b.prof_enable(True)

    # the warmup steps' gather statistics are not the timed ones
    gstats.update(rounds=0, streams=0, bytes=0, digest_mismatches=0, tail_ms=[])
    barrier()
    # the host share follows each step's own timeline (auto split): the next
    # step's host round trips are set so that the host side ends RIC_BENCH_MARGIN
    # ms (default 120: a host side that overruns costs the step its time, one
    # that ends early only a few frames) before the GPU side did in this step.  The warmup's
    # estimate alone left the two sides +-1 % apart from step to step.
    margin = float(os.environ.get("RIC_BENCH_MARGIN", "120"))
    per_step = []

    def rebalance():
        nonlocal n_host, nstep
        th, tg = b.hybrid_times()
        nh = n_host
        if th > 0 and tg > 0 and n_host > 0:
            t_eff = th / (n_host / threads)           # host wall ms per round trip per thread, this step
            want = threads * (tg - margin) / t_eff
            nh = int(round(0.5 * n_host + 0.5 * want))
            nh = max(threads, min(nh, host_frames_room(a, threads), nfr - n_gpu))
        nh = int(allreduce(nh, "min"))
        n_host = nh
        nstep = n_host + n_gpu

    dsync()
    t0 = time.perf_counter()
    frames_timed = 0
    for i in range(a.steps):
        step()
        frames_timed += nstep
        per_step.append(nstep)
        if auto and i + 1 < a.steps:
            rebalance()
        progress("step %d/%d" % (i + 1, a.steps))
    dsync()
    dt = time.perf_counter() - t0
    barrier()
    dt = allreduce(dt, "max")

    # ---- the forward levels alone (rank 0, right after timing, before the
    # verification leaves the GPU idle for ~20 s and its clocks ramp down): in
    # the timed region the host frames' levels share the CUs with the stream
    # coder's waves.  Outputs to buffers of their own (the verification reads
    # the last step's decoded frames).
    iso = None
    prof_timed = b.prof_read() if b is not None else {}       # the timed region's stage timers (prof_enable resets them)
    if rank == 0 and b is not None and hybrid:
        bmi = wavelet_bytes(W, H)
        nlev_i = len(bmi["dwt"])
        l0_bytes_i = bmi["dwt"][0] + bmi["quant"][0]
        enc_bytes_i = sum(bmi["dwt"]) + sum(bmi["quant"]) + bmi["ll"]
        # the forward levels back to back, as in the step's front (the full
        # encode + decode + pixel loop, ric_batch_diag_gpu, put level 0 at
        # 0.91-1.08 ms per launch against 0.86 in the front: rocprofv3 kernel
        # trace of the round-6 HEAD bench, profiles/r06_head_kernel_stats.csv)
        b.prof_enable(False)
        b.diag_gpu_encode(frames[:slots], a.q, a.trans, 5)
        b.prof_enable(True)
        b.diag_gpu_encode(frames[:slots], a.q, a.trans, 10)
        pi = b.prof_read()
        if pi["fwd_l0"][1]:
            t_iso = pi["fwd_l0"][0] / pi["fwd_l0"][1]
            ach = l0_bytes_i / (t_iso * 1e-3) / 1e9
            fi = [pi["fwd_l%d" % l][0] / pi["fwd_l%d" % l][1] for l in range(nlev_i) if pi["fwd_l%d" % l][1]]
            we = _frac(sum(fi), enc_bytes_i)
            iso = {"avg_launch_ms": round(sum(fi) * slots, 4), "achieved": we.get("GBps"), "frac": we.get("frac"),
                   "level0": {"avg_launch_ms": round(pi["fwd_l0"][0] / pi["fwd_l0"][2], 4), "achieved": round(ach, 1),
                              "frac": round(ach / HBM_PEAK_GBS, 4)},
                   "per_level_us_per_frame": [round(x * 1e3, 2) for x in fi],
                   "gpu_wavelet_encode": we,
                   "note": "the forward levels alone, back to back as in the step's front "
                           "(ric_batch_diag_gpu_encode), %d frames per launch, 10 iterations after 5 untimed ones, "
                           "right after the timed region (before the verification)" % slots}
        b.prof_enable(False)

    # ---- verification (outside the timed region): EVERY frame of the last
    # step -- its .ric file and its decoded pixels -- against the reference
    # (oracle/_ref, the port when absent) run on that frame's input; rank 0's
    # frame 0 also against the reference's golden SHA-256
    verified, vnote = None, "skipped"
    if not a.no_verify:
        ok = True
        notes = []
        if b is not None:
            nd = min(nstep, a.distinct)
            exp, t_or, kind = oracle_expectations([frames[d].numpy() for d in range(nd)], a.q, a.trans, threads)
            bad = []
            got_dig = digests.numpy()
            for d in range(nd):
                want_dig = pixel_digest(exp[d][1])
                if not np.array_equal(outs_d[d % nout].numpy(), exp[d][1].reshape(CH, H, W)):
                    bad.append(d)                  # the buffer's last writer, compared in full
                for k in range(d, nstep, a.distinct):
                    if b.stream(k) != exp[d][0] or got_dig[k] != want_dig:
                        bad.append(k)
            ok &= not bad
            ngpu = nstep - n_host if hybrid else 0
            notes.append("%d/%d frames of the last step (%d GPU-stream-coded, %d host-coded): .ric bytes and decoded "
                         "pixels (64-bit digest per frame, ric_batch_set_digests) equal the %s's on each frame's input (%d distinct inputs, %.1f s on %d threads)"
                         % (nstep - len(bad), nstep, ngpu, nstep - ngpu, "reference (oracle/_ref)" if kind == "reference"
                            else "oracle port", nd, t_or, threads))
            if bad:
                notes.append("mismatching frames %s" % bad[:16])
            gold = json.load(open(os.path.join(REPO, "tests", "golden", "golden.json")))["large"]
            want = None
            if a.q == 9 and a.trans == 0:
                if a.workload == "C3" and mine[0][1] == 0:
                    want = "C3_7680x4320_q9"
                elif a.workload == "C5" and mine[0][1] in (0, 1):
                    want = {0: "C2_4096x4096_q9", 1: "C5_frame1_4096x4096_q9"}[mine[0][1]]
                elif a.workload == "C4":
                    tx, ty = mine[0][2][0], mine[0][2][1]
                    want = "C4_tile_%d_%d" % (tx, ty)
            if want:
                e = [g for g in gold if g["name"] == want][0]
                ok &= hashlib.sha256(b.stream(0)).hexdigest() == e["ric_sha256"]
                ok &= hashlib.sha256(outs[0].numpy().tobytes()).hexdigest() == e["decoded_sha256"]
                notes.append("frame 0: %s golden sha256" % want)
        if gath is not None and rank == 0:
            ok &= gstats["digest_mismatches"] == 0
            notes.append("gather: %d streams (%d bytes) at rank 0 over the timed steps, %d digest mismatches"
                         % (gstats["streams"], gstats["bytes"], gstats["digest_mismatches"]))
        if world > 1:
            ok = bool(allreduce(1 if ok else 0, "min"))
            notes.append("%d ranks, %d frames in all" % (world, int(allreduce(nstep, "sum"))))
        verified, vnote = bool(ok), "; ".join(notes)
        if not ok:
            print(json.dumps({"error": "bench output mismatch", "rank": rank, "checked": vnote}), file=sys.stderr)
            sys.exit(3)

    # ---- stage timers (HIP events on the batch stream; host clocks)
    prof = prof_timed
    per_frame = {k: v[0] / v[1] for k, v in prof.items() if v[1]}
    per_launch = {k: v[0] / v[2] for k, v in prof.items() if v[2]}
    bm = wavelet_bytes(W, H)
    nlev = len(bm["dwt"])
    l0_bytes = bm["dwt"][0] + bm["quant"][0]
    fwd = [per_frame.get("fwd_l%d" % l) for l in range(nlev)]
    inv = [per_frame.get("inv_l%d" % l) for l in range(nlev)]
    enc_bytes = sum(bm["dwt"]) + sum(bm["quant"]) + bm["ll"]
    dec_bytes = sum(bm["dwt"]) + sum(bm["deq"])
    enc_ms = sum(fwd) if all(fwd) else None
    dec_ms = sum(inv) if all(inv) else None
    t_l0 = per_frame.get("fwd_l0")
    achieved = l0_bytes / (t_l0 * 1e-3) / 1e9 if t_l0 else None
    # the whole 5-level encode (DWT + quantiser over every
    # level, the headline roofline): the model bytes of a frame over the sum of
    # its level launches' per-frame times
    enc_achieved = enc_bytes / (enc_ms * 1e-3) / 1e9 if enc_ms else None
    traffic = traffic_enc = None
    pmc = os.path.join(REPO, "profiles", "pmc_fwd_l0_batch.json")
    if os.path.exists(pmc):
        try:
            p = json.load(open(pmc))
            if p.get("kernel", "").startswith("k_fwdq_pc_z") and p.get("W") == W and p.get("H") == H:
                traffic = p.get("hbm_bytes_per_frame")
        except Exception:
            traffic = None
    pmc_all = os.path.join(REPO, "profiles", "pmc_fwd_levels_batch.json")
    if os.path.exists(pmc_all):
        try:
            p = json.load(open(pmc_all))
            if p.get("W") == W and p.get("H") == H:
                traffic_enc = p.get("hbm_bytes_per_frame_all_levels")
        except Exception:
            traffic_enc = None
    # the pool / host payload compaction and the pool's expansion (compact.hip):
    # GPU work of this path outside the wavelet model.  Model bytes per frame:
    # compaction reads level 0's three dense 16-bit bands and their block
    # records (the value stream it writes is not counted); the expansion
    # writes the dense bands and reads the block masks (its values not counted)
    l0c = sum(((bx + 3) // 4) * ((by + 3) // 4) for bx, by in
              ((W // 2, H // 2), (W // 2, H // 2), (W // 2, H // 2)))
    l0coef = 3 * (W // 2) * (H // 2)
    cmp_bytes = 2 * l0coef + 8 * l0c
    dexp_bytes = 2 * l0coef + 2 * l0c

    # ---- the stream coder's launches (per launch: kernel time = a wave's time
    # to code one whole stream, with every stream of the launch in flight)
    coder = None
    if hybrid:
        coder = {"streams_per_launch": b.cp_pool, "frames_host_round_trip": n_host}
        # the coder's issue counters (SQ_INSTS_SALU / VALU, SQ_WAIT_ANY, ... per stream)
        # cannot be read inside this process: rocprofv3 --pmc over one serving step
        # of this path at C3 (scripts/gpu_sq.sh), committed under profiles/
        sqf = os.path.join(REPO, "profiles", "r06_stream_coder_sq.json")
        if not os.path.exists(sqf):
            sqf = os.path.join(REPO, "profiles", "r05_stream_coder_sq.json")
        if not os.path.exists(sqf):
            sqf = os.path.join(REPO, "profiles", "r04_stream_coder_sq.json")
        if os.path.exists(sqf) and a.workload == "C3":
            try:
                sq = json.load(open(sqf))
                rn = sq.get("default_run", "r4g_v2")
                run = sq["runs"][rn]
                coder["issue"] = {k: run[k] for k in ("kernel_s", "SQ_INSTS_SALU", "SQ_INSTS_VALU", "salu_share",
                                                       "instr_per_simd_per_4_cycles", "salu_per_cu_cycle", "wait_frac")
                                  if k in run}
                coder["issue"]["source"] = "profiles/%s runs.%s (per stream, %d streams in one k_gc_roundtrip " \
                                           "launch)" % (os.path.basename(sqf), rn, run.get("streams", sq["streams"]))
            except (OSError, ValueError, KeyError):
                pass
        if balance:
            coder["balance"] = balance
        for k, name in (("gpu_enc", "encode"), ("gpu_dec", "decode"), ("gpu_rt", "encode_then_decode")):
            if k in per_launch:
                ms, fr, ln = prof[k]
                coder[name] = {"launches": ln, "streams": fr, "ms_per_launch": round(ms / ln, 1),
                               "streams_per_s": round(fr / (ms * 1e-3), 1)}

    # ---- one frame's latency through ric_codec (rank 0, after timing): the
    # serial stage on one thread, and with the bands modelled in parallel
    lat = None
    if rank == 0 and b is not None and not a.no_latency:
        c = ric_amd.Codec(W, H, CH)
        want = b.stream(0)
        enc, same = {}, True
        for nt in sorted({1, 4, threads}):
            c.set_host_threads(nt)
            ts = []
            for _ in range(4):
                dsync()
                t0 = time.perf_counter()
                r = c.compress(frames[0], a.q, a.trans, on_device=True)
                ts.append(time.perf_counter() - t0)
                same = same and r == want
            enc[str(nt)] = round(float(np.median(ts[1:])) * 1e3, 2)
        td = []
        for _ in range(4):
            dsync()
            t0 = time.perf_counter()
            c.decompress(want, pix_out=outs[0])
            dsync()
            td.append(time.perf_counter() - t0)
        lat = {"encode_ms_by_host_threads": enc, "decode_ms": round(float(np.median(td[1:])) * 1e3, 2),
               "bytes_equal_step_frame0": bool(same),
               "note": "one %dx%dx%d frame through ric_codec (CompressImage / DecompressImage), pixels and decoded "
                       "output in HBM, median of 3 after one warm call, after the timed region; host threads n: the "
                       "bands of a plane modelled on n - 1 pool threads while the calling thread writes the stream "
                       "(ric_codec_set_host_threads); the decoder is serial" % (W, H, CH)}
        del c
        if not same:
            print(json.dumps({"error": "latency codec output differs from the step's frame 0"}), file=sys.stderr)
            sys.exit(3)

    # ---- encode-only and decode-only rates of the same path (rank 0, after timing)
    split = None
    if rank == 0 and b is not None and not a.no_split and not hybrid:
        streams = [b.stream(i) for i in range(nfr)]
        dsync()
        te = time.perf_counter()
        for g in range(0, nfr, slots):
            b.compress(frames[g:g + slots], a.q, a.trans, on_device=True)
        te = time.perf_counter() - te
        td = time.perf_counter()
        for g in range(0, nfr, slots):
            b.decompress(streams[g:g + slots], pix_out=outs[g:g + slots])
        dsync()
        td = time.perf_counter() - td
        mpx = nfr * W * H / 1e6
        split = {"encode_mpix_s": round(mpx / te, 2), "decode_mpix_s": round(mpx / td, 2),
                 "note": "rank 0, %d frames in groups of %d, groups not pipelined" % (nfr, slots)}

    total_px = frames_timed * W * H                 # every timed step's frames (the auto split varies them)
    sum_px = allreduce(total_px, "sum")
    value = sum_px / 1e6 / dt
    wl = {"C3": "C3: 7680x4320 gray, 5-level cdf97, q=%d, .ric encode+decode round trip, bit-exact" % a.q,
          "C5": "C5: %d x 4096x4096 gray frames per step, 5-level cdf97, q=%d, encode+decode, frame f on rank f mod N"
                % (a.frames or a.batch or 64, a.q),
          "C4": "C4: 7680x4320 RGB as 2x2 tiles of 3840x2160, q=%d, encode+decode, tile (tx,ty) on rank 2ty+tx, "
                "RCCL gather of the tile streams" % a.q}[a.workload]
    hs = None
    if a.workload == "C3" and a.q == 9 and a.trans == 0 and per_frame.get("host_enc"):
        hs = {"events_per_frame": C3_EVENTS,
              "encode_Mevents_s_per_thread": round(C3_EVENTS / per_frame["host_enc"] / 1e3, 1),
              "decode_Mevents_s_per_thread": round(C3_EVENTS / per_frame["host_dec"] / 1e3, 1),
              "note": "reference codeBin + bitsCode call count of a C3 frame (SURVEY.md §6) over this path's host "
                      "coder time per frame; the survey's replay of those events through CMuxCodec alone: 216 "
                      "Mevents/s on one core"}
    out = {
        "metric": "encode+decode Mpixel/s on 8K gray, 5-level wavelet; % HBM roofline",
        "value": round(value, 2),
        "unit": "Mpixel/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic (SURVEY.md §8(d) generator), resident in HBM",
        "config": {"workload": wl, "frames_per_gpu_per_step": (nstep if len(set(per_step)) <= 1 else round(frames_timed / a.steps, 2)),
                   "frames_per_step_timed": per_step, "frames_per_launch": slots,
                   "host_coder_threads_per_gpu": threads, "parallelism": "frames sharded over %d GPU(s)" % world,
                   "coder": ("GPU stream coder (one wave per stream, %d streams per launch): encode%s of %d of %d "
                             "frames; host threads: %s" % (b.cp_pool, {0: "", 1: " and decode", 2: " (and decode of the "
                                                                        "launches the host threads have no room for)"}[gpu_dec],
                                                           nstep - n_host, nstep,
                                                           {0: "round trips of the rest and every decode",
                                                            1: "round trips of the rest",
                                                            2: "round trips of the rest and the decode of the other "
                                                               "launches"}[gpu_dec])) if hybrid
                   else "host threads (encode and decode)"},
        "verified": verified,
        "verified_against": vnote,
        "roofline": {"bound": "hbm",
                     "kernel": "the 5-level forward wavelet encode (SURVEY.md §8(d) DWT + quantiser): k_fwdq_pc_z "
                               "level 0, k_fwdq_pc2_z levels 1-2, k_fwdq_gen_z levels 3-4 (+ LL TSUQ), fused DWT + "
                               "RD quantiser + block records, %d frames per launch; per launch = the five level "
                               "launches of one group" % slots,
                     "achieved": round(enc_achieved, 1) if enc_achieved else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(enc_achieved / HBM_PEAK_GBS, 4) if enc_achieved else None,
                     "traffic": traffic_enc * slots if traffic_enc else None,
                     "algorithmic_bytes_per_launch": enc_bytes * slots,
                     "avg_launch_ms": round(enc_ms * slots, 4) if enc_ms else None,
                     "level0": {"kernel": "k_fwdq_pc_z level 0", "achieved": round(achieved, 1) if achieved else None,
                                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                                "traffic": traffic * slots if traffic else None,
                                "algorithmic_bytes_per_launch": l0_bytes * slots,
                                "avg_launch_ms": round(per_launch["fwd_l0"], 4) if "fwd_l0" in per_launch else None}},
        "gpu_wavelet_encode": _frac(enc_ms, enc_bytes),
        "gpu_wavelet_decode": _frac(dec_ms, dec_bytes),
        "compaction": {"write": _frac(per_frame.get("compact"), cmp_bytes),
                       "expand": _frac(per_frame.get("dcmp_expand"), dexp_bytes),
                       "vs_level0": round((per_frame.get("compact", 0) + per_frame.get("dcmp_expand", 0)) / t_l0, 3)
                       if t_l0 else None,
                       "note": "k_cmp_count/scan/write (pool frames and host frames) and k_dcmp_expand, per frame "
                               "they ran on; bytes: the dense level-0 bands + block records (masks) they read or "
                               "write, value streams not counted; vs_level0: their time over level 0's"},
        "per_level_us_per_frame": {"fwd": [round(x * 1e3, 2) if x else None for x in fwd],
                                   "inv": [round(x * 1e3, 2) if x else None for x in inv]},
        "stage_ms_per_frame": {k: round(v, 4) for k, v in per_frame.items()},
        "bytes_per_frame": int(np.mean([len(b.stream(i)) for i in range(nstep)])) if b is not None else None,
    }
    if hs:
        out["host_serial"] = hs
    if split:
        out["gpu_path_split"] = split
    if coder:
        out["stream_coder"] = coder
    if iso:
        out["roofline_isolated"] = iso
    if lat:
        out["latency"] = lat
    if gather:
        out["gather"] = {"backend": backend, "bytes_to_rank0_per_step": gathered[0] // max(a.steps, 1)
                         if a.workload != "C4" else gathered[0]}
        if gath is not None:
            out["gather"].update({
                "streams_to_rank0_per_step": gstats["streams"] // max(a.steps, 1),
                "rounds_per_step": gstats["rounds"] / max(a.steps, 1),
                "digest_mismatches": gstats["digest_mismatches"],
                "chunk_bytes": gath.chunk,
                "rank0_gather_buffers_bytes": (world - 1) * gath.chunk,
                "finish_after_coding_ms": gstats["tail_ms"],
                "note": "every stream of every rank, shipped in chunks of at most chunk_bytes while the step runs "
                        "(a stream leaves once its .ric file is complete), digest-checked at rank 0; "
                        "finish_after_coding_ms: how long after this rank's coding the gather ended, per timed step"})
        if a.workload == "C4":
            out["gather"]["container"] = "RTL1, 4 tiles, %d bytes; tiles scattered back per step" % gathered[0]
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(W, H, a.q, a.trans, threads)   # gray frames of the workload's size
        except Exception as e:
            out["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out))
    del b
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
