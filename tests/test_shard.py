"""Frame/tile sharding and the stream gather (rududu-image-codec_amd/shard.py):
host logic plus a world_size-2 gloo run (the GPU runs use the same code with
the nccl=RCCL backend)."""
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


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "rududu-image-codec_amd"))
    import torch.distributed as dist
    import shard as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = S.frames_of_rank(7, world, rank)
    local = [(b"frame%d:" % f) * (f + 1) for f in frames]
    res = S.gather_streams(local, dist)
    dev = S.gather_streams(local, dist, to_host=False)   # bench.py's form
    if dev is not None:
        bufs, szs = dev
        dev = [[bytes(b[int(s[1:1 + i].sum()):int(s[1:2 + i].sum())].numpy()) for i in range(int(s[0]))]
               for b, s in zip(bufs, szs)]
    q.put((rank, (res, dev)))
    dist.destroy_process_group()


def test_gather_streams_gloo_world2():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    assert out[1] == (None, None)
    got, got_dev = out[0]
    assert got_dev == got
    assert [len(x) for x in got] == [4, 3]
    flat = {}
    for r, lst in enumerate(got):
        for f, s in zip(shard.frames_of_rank(7, 2, r), lst):
            flat[f] = s
    assert all(flat[f] == (b"frame%d:" % f) * (f + 1) for f in range(7))


def _worker_tiles(rank, world, port, q):
    """C4's exchange: each rank's tile streams to rank 0 (gather), the RTL1
    container there, and the decode side: unpack + scatter back."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "rududu-image-codec_amd"))
    import torch.distributed as dist
    import shard as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = S.tiles_of_rank(world, rank)
    local = [(b"tile%d|" % i) * (50 + 7 * i) for i in mine]
    got = S.gather_streams(local, dist)
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
    mine_back = S.scatter_streams(per_rank, dist)
    q.put((rank, (local, mine_back, blob)))
    dist.destroy_process_group()


def test_tiles_gather_container_scatter_gloo_world2():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_tiles, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    for r in range(2):
        local, back, _ = out[r]
        assert back == local and len(local) == 2
    W, H, nx, ny, streams = shard.unpack_tiles(out[0][2])
    assert (W, H, nx, ny) == (7680, 4320, 2, 2)
    assert streams == [(b"tile%d|" % i) * (50 + 7 * i) for i in range(4)]
