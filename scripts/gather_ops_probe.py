#!/usr/bin/env python3
"""gather_ops_probe.py -- each stream-gather device operation timed on its own
while a 3072-stream coder launch (three coder waves on every SIMD) is in
flight: which of them, if any, waits for the launch.  Development tool (GPU
box); RIC_AMD_LIB selects a library build, PROBE_N the stream count."""
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rududu-image-codec_amd"))


def main():
    import ric_amd as ric
    import shard
    w, h = 2048, 1088
    n = int(os.environ.get("PROBE_N", "3072"))
    pool = n // 2
    distinct = 8
    dev = [ric.DeviceArray.from_numpy(ric.synth(w, h, 1, 700 + i)) for i in range(distinct)]
    frames = [dev[i % distinct] for i in range(n)]
    pouts = [ric.DeviceArray((1, h, w), np.uint8) for _ in range(distinct)]
    outs = [pouts[i % distinct] for i in range(n)]
    scap = (w * h * 3 // 8 + 65536) // 16 * 16
    b = ric.Batch(w, h, 1, slots=16, threads=2)
    b.hybrid_config(pool, scap)
    words = np.zeros(n, np.uint32)
    b.set_ready(words, n)
    sbufs = [np.empty(scap, np.uint8) for _ in range(n)]
    comm = ric.Comm(ric.Comm.unique_id(), 1, 0, 0)
    t = shard.RcclTransport(comm, 0)
    chunk = np.random.default_rng(9).integers(0, 256, 4 << 20, dtype=np.uint8)
    dchunk = ric.DeviceArray.from_numpy(chunk)
    back = ric.DeviceArray(1 << 20, np.uint8, zero=True)
    pin = ric.pinned_array(1 << 20)
    ops = [("digests", lambda: ric.device_digests(0, dchunk, [0, 1 << 20], [1 << 20, 1 << 20])),
           ("h2d_pageable", lambda: t.put(back, 0, chunk[:1 << 20])),
           ("d2h_pageable", lambda: back.numpy()),
           ("d2h_pinned", lambda: ric._chk(ric.lib().ric_device_copy(0, pin.ctypes.data, back.data_ptr(), 1 << 20,
                                                                      ric.RIC_COPY_D2H), "d2h")),
           ("pack_h2d", lambda: t.put_many(back, [chunk[:1000], chunk[5000:7000]], [0, 1008])),
           ("rccl_self", lambda: comm.sendrecv([(0, True, dchunk, 1 << 20), (0, False, back, 1 << 20)]))]
    for name, f in ops:                      # warm
        f()
    for rep in range(2):
        words[:] = 0
        err = []

        def run():
            try:
                b.roundtrip_hybrid(frames, outs, 0, 9, 0, gpu_decode=1, streams=sbufs)
            except Exception as e:
                err.append(e)
        th = threading.Thread(target=run)
        t0 = time.perf_counter()
        th.start()
        while not words.any():
            time.sleep(0.001)
        t_first = time.perf_counter() - t0
        res = []
        for name, f in ops:
            a = time.perf_counter()
            f()
            res.append((name, round((time.perf_counter() - a) * 1e3, 2), th.is_alive()))
        tl = []
        if os.environ.get("PROBE_TL"):
            # RCCL availability over the rest of the launch: one 1 MiB
            # self send/receive every ~10 ms, (ms into the launch, its latency)
            while th.is_alive():
                a = time.perf_counter()
                comm.sendrecv([(0, True, dchunk, 1 << 20), (0, False, back, 1 << 20)])
                tl.append((round((a - t0) * 1e3), round((time.perf_counter() - a) * 1e3, 1)))
                time.sleep(0.01)
        th.join()
        if tl:
            print("  rccl timeline (ms into launch, latency ms):", tl, flush=True)
        print("rep %d: launch %.0f ms, first ready %.0f ms: %s%s" % (rep, (time.perf_counter() - t0) * 1e3, t_first * 1e3,
                                                                   res, " ERR %s" % err if err else ""), flush=True)


if __name__ == "__main__":
    main()
