"""Frame/tile sharding and the stream gather (rududu-image-codec_amd/shard.py):
host logic plus multi-process gloo runs of the gather protocol (the GPU runs
use the same StreamGather over the library's RCCL communicator)."""
import os
import socket

import numpy as np
import pytest

import shard


def test_frames_partition():
    for world in (1, 2, 4, 8):
        got = sorted(sum((shard.frames_of_rank(64, world, r) for r in range(world)), []))
        assert got == list(range(64))
        assert all(len(shard.frames_of_rank(64, world, r)) == 64 // world for r in range(world))


def test_tiles_partition():
    for world in (1, 2, 3, 4):
        got = sorted(sum((shard.tiles_of_rank(world, r) for r in range(world)), []))
        assert got == [0, 1, 2, 3]
    assert [shard.tiles_of_rank(4, r) for r in range(4)] == [[0], [1], [2], [3]]
    assert [shard.tile_of_rank(r) for r in range(4)] == [shard.tile_rects(8, 8)[r][:2] for r in range(4)]


def test_bench_workload_partition():
    """bench.py's C3 / C4 / C5 frame sets: every frame or tile exactly once
    over the ranks."""
    import argparse
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    for wl in ("C4", "C5"):
        for world in (1, 2, 4, 8):
            a = argparse.Namespace(workload=wl, frames=0, batch=0)
            seen = []
            for r in range(world):
                W, H, C, mine, scaling = bench.workload_frames(a, r, world, 16)
                seen += [m[0] for m in mine]
                assert scaling == "strong"
            assert sorted(seen) == list(range(4 if wl == "C4" else 64))
    a = argparse.Namespace(workload="C3", frames=0, batch=0)
    f0 = bench.workload_frames(a, 0, 2, 16)[3]
    f1 = bench.workload_frames(a, 1, 2, 16)[3]
    assert len(f0) == len(f1) == 128 and not set(m[1] for m in f0) & set(m[1] for m in f1)


def test_tiles_cover_image():
    rects = shard.tile_rects(7680, 4320)
    assert [(r[0], r[1]) for r in rects] == [(0, 0), (1, 0), (0, 1), (1, 1)]
    cov = np.zeros((4320, 7680), np.int32)
    for (_, _, x0, y0, w, h) in rects:
        cov[y0:y0 + h, x0:x0 + w] += 1
    assert (cov == 1).all()
    assert rects[3][2:] == (3840, 2160, 3840, 2160)
    odd = shard.tile_rects(1001, 603)
    assert sum(r[4] * r[5] for r in odd) == 1001 * 603


def test_tile_container_roundtrip():
    streams = [bytes([i]) * (10 + i) for i in range(4)]
    blob = shard.pack_tiles(7680, 4320, 2, 2, streams)
    W, H, nx, ny, got = shard.unpack_tiles(blob)
    assert (W, H, nx, ny) == (7680, 4320, 2, 2) and got == streams
    with pytest.raises(ValueError):
        shard.unpack_tiles(b"RUD2....")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "rududu-image-codec_amd"))
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _stream(rank, i):
    rng = np.random.default_rng(1000 * rank + i)
    return rng.integers(0, 256, int(rng.integers(1, 9000)), dtype=np.uint8).tobytes()


def _worker_gather(rank, world, port, nper, q):
    """Every rank codes nper[rank] streams that become ready in a random
    order over time (a producer thread sets their ready words, as
    ric_batch_set_ready does); they are shipped in 16 KiB chunks."""
    import threading
    import time
    dist = _init(rank, world, port)
    import shard as S
    t = S.GlooTransport(dist)
    g = S.StreamGather(t, rank, world, chunk_bytes=16 << 10)
    n = nper[rank]
    streams = [_stream(rank, i) for i in range(n)]
    if rank == 0:
        got = {}
        g.receive(lambda r, i, b: got.__setitem__((r, i), bytes(b)))
        held = sum(b.size for b in g.bufs) + sum(h.size for h in g.hdr)
        q.put((rank, (got, g.stats, held)))
    else:
        words = np.zeros(n, np.uint32)
        order = np.random.default_rng(rank).permutation(n)

        def produce():
            for k, i in enumerate(order):
                words[i] = len(streams[i])
                if k % 7 == 0:
                    time.sleep(0.002)
        th = threading.Thread(target=produce)
        th.start()
        st = g.send(n, words, lambda i, ln: streams[i])
        th.join()
        q.put((rank, st))
    dist.destroy_process_group()


def _spawn(target, world, *args):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    return out


@pytest.mark.parametrize("world,nper", [(2, [0, 150]), (3, [5, 97, 0])])
def test_stream_gather_gloo(world, nper):
    """Every stream of every rank arrives at rank 0 byte-exact (digests
    checked on arrival), in bounded chunks: rank 0 holds one 16 KiB chunk per
    peer however many streams there are."""
    out = _spawn(_worker_gather, world, nper)
    got, stats, held = out[0]
    assert stats["digest_mismatches"] == []
    for r in range(1, world):
        assert stats["streams"][r] == nper[r] == out[r]["streams"]
        for i in range(nper[r]):
            assert got[(r, i)] == _stream(r, i), (r, i)
    assert len(got) == sum(nper[1:])
    assert held <= (world - 1) * ((16 << 10) + 8 * 196 + 64)
    if nper[1] > 64:
        assert stats["rounds"] > 2             # many streams: several chunks


def _worker_tiles(rank, world, port, q):
    """C4's exchange: each rank's tile streams to rank 0 (gather), the RTL1
    container there, and the decode side: unpack + scatter back."""
    dist = _init(rank, world, port)
    import shard as S
    t = S.GlooTransport(dist)
    mine = S.tiles_of_rank(world, rank)
    local = [(b"tile%d|" % i) * (50 + 7 * i) for i in mine]
    got = S.gather_streams(local, t, rank, world)
    blob = None
    per_rank = None
    if rank == 0:
        streams = [None] * 4
        for r, lst in enumerate(got):
            for i, s in zip(S.tiles_of_rank(world, r), lst):
                streams[i] = s
        blob = S.pack_tiles(7680, 4320, 2, 2, streams)
        _, _, _, _, back = S.unpack_tiles(blob)
        per_rank = [[back[i] for i in S.tiles_of_rank(world, r)] for r in range(world)]
    mine_back = S.scatter_streams(per_rank, t, rank, world)
    q.put((rank, (local, mine_back, blob)))
    dist.destroy_process_group()


def test_tiles_gather_container_scatter_gloo_world2():
    out = _spawn(_worker_tiles, 2)
    for r in range(2):
        local, back, _ = out[r]
        assert back == local and len(local) == 2
    W, H, nx, ny, streams = shard.unpack_tiles(out[0][2])
    assert (W, H, nx, ny) == (7680, 4320, 2, 2)
    assert streams == [(b"tile%d|" % i) * (50 + 7 * i) for i in range(4)]


def test_digest_matches_device_formula():
    """shard.digest_bytes is ric_batch_set_digests' formula (bench.py
    pixel_digest), which the device digest kernel implements"""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    a = np.random.default_rng(3).integers(0, 256, 100003, dtype=np.uint8)
    assert shard.digest_bytes(a) == bench.pixel_digest(a)


def test_host_digests_native():
    """ric_host_digests (the gloo transport's and the RCCL sender's digest) is
    the same formula: runs longer than its 4096-byte blocks, odd offsets,
    empty runs."""
    import ric_amd
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, 300000, dtype=np.uint8)
    buf[1000:20000] = 255                     # the 32-bit block sums at their largest
    offs = [0, 1, 17, 4095, 4096, 8191, 100, 0]
    lens = [0, 1, 5000, 4097, 70000, 123456, 19000, 300000]
    got = ric_amd.host_digests(buf, offs, lens)
    want = [shard.digest_bytes(buf[o:o + n]) for o, n in zip(offs, lens)]
    assert [int(x) for x in got] == [int(x) for x in want]


def test_put_many_packs_and_digests():
    t = shard.GlooTransport(None)
    buf = t.alloc(1 << 16)
    buf[:] = 7
    srcs = [b"abc", np.arange(100, dtype=np.uint8), b"", b"xyz" * 50]
    offs = [0, 16, 128, 128]
    dg = t.put_many(buf, srcs, offs)
    assert bytes(buf[:3]) == b"abc" and not buf[3:16].any()
    assert np.array_equal(buf[16:116], np.arange(100, dtype=np.uint8)) and not buf[116:128].any()
    assert bytes(buf[128:278]) == b"xyz" * 50
    assert [int(x) for x in dg] == [int(shard.digest_bytes(np.frombuffer(s, np.uint8) if isinstance(s, bytes) else s))
                                    for s in srcs]


def _worker_big(rank, world, port, q):
    """gather_streams with a peer whose streams are larger than rank 0's (and
    than 1 MiB), empty streams included; scatter_streams of more than 64
    streams per rank."""
    dist = _init(rank, world, port)
    import shard as S
    t = S.GlooTransport(dist)
    rng = np.random.default_rng(rank)
    sizes = {0: [100, 0], 1: [3 << 20, 0, 1500000, 7], 2: [0]}[rank]
    local = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in sizes]
    got = S.gather_streams(local, t, rank, world)
    per_rank = None
    if rank == 0:
        per_rank = [[bytes([r, i % 256]) * (i % 5) for i in range(70 + r)] for r in range(world)]
    back = S.scatter_streams(per_rank, t, rank, world)
    q.put((rank, (local, got, back)))
    dist.destroy_process_group()


def test_gather_big_and_empty_streams_scatter_many_gloo():
    out = _spawn(_worker_big, 3)
    got = out[0][1]
    assert [g for g in got] == [out[r][0] for r in range(3)]
    for r in range(3):
        assert out[r][2] == [bytes([r, i % 256]) * (i % 5) for i in range(70 + r)]


def test_gather_rejects_oversized_chunk_header():
    """Rank 0 grows a peer's buffer to the payload size its header announces,
    up to StreamGather.max_chunk: a corrupt header asking for more is refused
    before any allocation."""
    class OneHeader(shard.GlooTransport):
        def __init__(self, size):
            super().__init__(None)
            self.size = size
            self.allocs = []

        def alloc(self, nbytes):
            self.allocs.append(int(nbytes))
            return super().alloc(nbytes)

        def sendrecv(self, ops):
            for peer, is_send, buf, n in ops:
                assert not is_send
                if n == shard.HDR_WORDS * 8:
                    h = np.zeros(shard.HDR_WORDS, np.int64)
                    h[1], h[2], h[3] = 0, 1, self.size
                    buf[:n] = h.view(np.uint8)

    t = OneHeader(3 << 30)
    g = shard.StreamGather(t, 0, 2, chunk_bytes=1 << 20, max_chunk=1 << 24)
    with pytest.raises(RuntimeError, match="bad chunk header"):
        g.receive()
    assert max(t.allocs) <= 1 << 20
    ok = OneHeader(1 << 22)                    # within the bound: grown and accepted
    g = shard.StreamGather(ok, 0, 2, chunk_bytes=1 << 20, max_chunk=1 << 24)
    g.receive()
    assert g.cap[0] == 1 << 22
