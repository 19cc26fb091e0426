"""Operations beside a stream coder launch in flight (the gather's side of the
serving step): they must complete while the launch's waves still
run, not wait for the launch to end.

This file is collected last on purpose (its name): its bounds are wall-clock
bounds, so a regression here stops `pytest -x` only after every parity test
has run.  Each operation is timed on its own and the assertion message lists
them all, with any garbage collection that ran inside the window, so a failure
names the operation that waited.

Round 5's failure in the full suite (digests + copies + pack 722 ms = the rest
of the launch, passing alone) had this cause: a Batch of an earlier test,
held in a reference cycle by a `pytest.raises` traceback, was collected by
Python's cyclic GC inside the window, and its destructor's hipFree synchronises
every stream of the device -- the coder's launch included.  The library now
parks frees issued while a coder call runs (ric_device_free, every ric_*
destroy: include/ric_gpu.h) and frees them when the call ends; the second half
of the test destroys a Batch and a device buffer during the launch on purpose.
"""
import gc
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

OP_MS = 100.0          # one side-stream operation (digests, a 1 MiB copy, a pack, a free)
RCCL_MS = 50.0         # a one-rank send/receive after the first


def test_gather_ops_during_coder_launch(ric, port):
    """Once a 3072-stream k_gc_roundtrip (three coder waves on every SIMD, the
    serving step's load) has posted its first streams: device digests, H2D /
    D2H copies, a chunk pack, a one-rank RCCL send / receive, and the release
    of a device buffer and of a whole Batch all finish while the launch still
    runs.  Also prints rank 0's receive-side cost of one 64 MiB chunk of 64
    streams (digests + D2H into pinned memory), in flight and idle."""
    import shard
    w, h, n, pool = 2048, 1088, 3072, 1536
    distinct = 8
    host = [ric.synth(w, h, 1, 700 + i) for i in range(distinct)]
    dev = [ric.DeviceArray.from_numpy(x) for x in host]
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
    rng = np.random.default_rng(9)
    chunk = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
    dchunk = ric.DeviceArray.from_numpy(chunk)
    back = ric.DeviceArray(1 << 20, np.uint8, zero=True)
    offs = [i << 20 for i in range(64)]
    lens = [(1 << 20) - 16 * i for i in range(64)]
    want = [shard.digest_bytes(chunk[o:o + L]) for o, L in zip(offs, lens)]
    # released during the launch on purpose (second half)
    victims = {"batch": ric.Batch(256, 192, 1, slots=2, threads=1),
               "buffer": ric.DeviceArray(16 << 20, np.uint8)}
    victims["batch"].roundtrip([ric.DeviceArray.from_numpy(ric.synth(256, 192, 1, 3))],
                               [ric.DeviceArray((1, 192, 256), np.uint8)], q=9, trans=0)

    def rank0_chunk():
        t0 = time.perf_counter()
        dg = t.digests(dchunk, offs, lens)
        t1 = time.perf_counter()
        sink = t.get(dchunk, 0, 64 << 20)
        t2 = time.perf_counter()
        assert [int(x) for x in dg] == [int(x) for x in want]
        assert sink[12345] == chunk[12345]
        return (t1 - t0) * 1e3, (t2 - t1) * 1e3

    rank0_chunk()                                   # warm (pinned sink, scratch, staging)
    t.put_many(back, [chunk[:16]], [0])
    err = []

    def run():
        try:
            b.roundtrip_hybrid(frames, outs, 0, 9, 0, gpu_decode=1, streams=sbufs)
        except Exception as e:                      # pragma: no cover
            err.append(e)

    gc.collect()                                    # (the library no longer depends on it: see the second half)
    gcs = []

    def on_gc(phase, info):
        gcs.append("%s gen %s at %.1f ms" % (phase, info.get("generation"), (time.perf_counter() - t_start) * 1e3))
    gc.callbacks.append(on_gc)
    ops = []

    def timed(label, fn):
        t0 = time.perf_counter()
        r = fn()
        ops.append((label, (time.perf_counter() - t0) * 1e3))
        return r

    try:
        th = threading.Thread(target=run)
        t_start = time.perf_counter()
        th.start()
        while not words.any():
            assert th.is_alive(), err
            time.sleep(0.001)
        t_first = time.perf_counter() - t_start
        parked0 = ric.lib().ric_diag_deferred_frees()
        dg = timed("device digests", lambda: ric.device_digests(0, dchunk, offs[:4], lens[:4]))
        timed("H2D 1 MiB", lambda: t.put(back, 0, chunk[:1 << 20]))
        got = timed("D2H 1 MiB", back.numpy)
        pk = timed("chunk pack", lambda: t.put_many(back, [chunk[:1000], chunk[5000:7000]], [0, 1008]))
        # RCCL: the first send/receive of a launch may wait until the launch's
        # first waves retire; the next ones go straight through
        rccl_ms = []
        for k in range(2):
            t1 = time.perf_counter()
            comm.sendrecv([(0, True, dchunk.data_ptr() + ((k + 1) << 20), 1 << 20), (0, False, back, 1 << 20)])
            rccl_ms.append((time.perf_counter() - t1) * 1e3)
            assert np.array_equal(back.numpy(), chunk[(k + 1) << 20:(k + 2) << 20])
        busy = rank0_chunk()
        # the releases a garbage collector or a server's cleanup would make
        timed("free a device buffer", lambda: victims.pop("buffer").__del__())
        timed("destroy a Batch", lambda: victims.pop("batch").__del__())
        parked = ric.lib().ric_diag_deferred_frees() - parked0
        alive = th.is_alive()
        n_ready = int((words != 0).sum())
        th.join()
    finally:
        gc.callbacks.remove(on_gc)
    assert not err, err
    total = time.perf_counter() - t_start
    idle = rank0_chunk()
    report = ("launch %.0f ms, first stream ready at %.0f ms, %d of %d ready after the ops; %s; "
              "RCCL send/receive %.1f ms (first) / %.1f ms (next); %d frees parked; GC in the window: %s; "
              "rank-0 64 MiB chunk (digests ms, D2H ms): in flight %.1f / %.1f, idle %.1f / %.1f"
              % (total * 1e3, t_first * 1e3, n_ready, n, ", ".join("%s %.1f ms" % o for o in ops),
                 rccl_ms[0], rccl_ms[1], parked, gcs or "none", busy[0], busy[1], idle[0], idle[1]))
    print("\n[gather-ops] " + report)
    assert [int(x) for x in dg] == [int(x) for x in want[:4]], report
    assert np.array_equal(got, chunk[:1 << 20]), report
    assert [int(x) for x in pk] == [int(shard.digest_bytes(chunk[:1000])), int(shard.digest_bytes(chunk[5000:7000]))]
    assert alive, "the coder launch ended before the operations did: " + report
    slow = [o for o in ops if o[1] >= OP_MS]
    assert not slow, "waited for the coder launch: %s | %s" % (slow, report)
    assert rccl_ms[1] < RCCL_MS, report
    assert parked >= 2, "the frees during the launch were not parked: " + report
    r = b.stream(0)
    assert r == port.encode_ric(host[0], 9, 0)
    # the parked buffers were freed when the call ended: a new allocation of
    # the same size and a fresh Batch still work
    again = ric.Batch(256, 192, 1, slots=2, threads=1)
    x = ric.synth(256, 192, 1, 3)
    o = ric.DeviceArray((1, 192, 256), np.uint8)
    again.roundtrip([ric.DeviceArray.from_numpy(x)], [o], q=9, trans=0)
    assert again.stream(0) == port.encode_ric(x, 9, 0)
