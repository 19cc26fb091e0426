"""Frame / tile sharding across GPUs and the gather of compressed .ric streams
(SURVEY.md §8(e)).

Independent frames (C5) and tiles (C4) are independent .ric streams, so ranks
share no state while coding: frame f goes to rank f mod N, tile (tx, ty) of a
2x2 grid to rank 2*ty + tx.  The only exchange is the final gather of the
variable-size compressed streams to rank 0: an all_gather of the stream sizes
(int64), then a gather of the size-padded payloads to rank 0 (RCCL over xGMI
with the "nccl" backend on GPUs, gloo on CPU).

Tile container ("RTL1", our extension -- the reference has no tile syntax):
  "RTL1" | u16 W | u16 H | u8 nx | u8 ny | nx*ny u32 LE stream sizes |
  the tile .ric files back to back, row-major (ty outer, tx inner).
Each tile is a standalone .ric of the crop (x0 = tile_w * tx, y0 = tile_h * ty).
"""
import struct

import numpy as np

TILE_MAGIC = b"RTL1"


def frames_of_rank(n_frames, world, rank):
    """Frame indices coded by `rank` (f mod world == rank)."""
    return list(range(rank, n_frames, world))


def tile_rects(W, H, nx=2, ny=2):
    """[(tx, ty, x0, y0, w, h)] row-major; the last row/column takes the remainder."""
    tw, th = W // nx, H // ny
    out = []
    for ty in range(ny):
        for tx in range(nx):
            w = tw if tx < nx - 1 else W - tw * (nx - 1)
            h = th if ty < ny - 1 else H - th * (ny - 1)
            out.append((tx, ty, tw * tx, th * ty, w, h))
    return out


def tile_of_rank(rank, nx=2, ny=2):
    return rank % nx, rank // nx


def tiles_of_rank(world, rank, nx=2, ny=2):
    """Tile indices (2*ty + tx for 2x2) coded by `rank`: tile i on rank i mod
    world -- one tile per rank at world == nx*ny, round robin
    below that."""
    return list(range(rank, nx * ny, world))


def pack_tiles(W, H, nx, ny, streams):
    assert len(streams) == nx * ny
    head = TILE_MAGIC + struct.pack("<HHBB", W, H, nx, ny) + struct.pack("<%dI" % len(streams),
                                                                        *[len(s) for s in streams])
    return head + b"".join(streams)


def unpack_tiles(blob):
    if blob[:4] != TILE_MAGIC:
        raise ValueError("not an RTL1 tile container")
    W, H, nx, ny = struct.unpack_from("<HHBB", blob, 4)
    n = nx * ny
    sizes = struct.unpack_from("<%dI" % n, blob, 10)
    off = 10 + 4 * n
    streams = []
    for s in sizes:
        streams.append(bytes(blob[off:off + s]))
        off += s
    return W, H, nx, ny, streams


def gather_streams(local, dist, device=None, to_host=True):
    """All ranks pass their list of byte streams; rank 0 gets every rank's
    list (in rank order), other ranks get None.  Two collectives: sizes, then
    the padded payloads.  to_host=False: rank 0 gets (payload tensors, size
    tensors) per rank as they arrived on `device` (size tensor = [n, len...])."""
    import torch
    world = dist.get_world_size()
    rank = dist.get_rank()
    dev = device if device is not None else torch.device("cpu")
    n_local = len(local)
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(counts, torch.tensor([n_local], dtype=torch.int64, device=dev))
    maxn = max(int(c[0]) for c in counts)
    sz = torch.zeros(maxn + 1, dtype=torch.int64, device=dev)
    sz[0] = n_local
    if n_local:
        sz[1:n_local + 1] = torch.tensor([len(x) for x in local], dtype=torch.int64, device=dev)
    all_sz = [torch.zeros_like(sz) for _ in range(world)]
    dist.all_gather(all_sz, sz)
    total = max(int(t[1:].sum()) for t in all_sz)
    buf = torch.zeros(max(total, 1), dtype=torch.uint8, device=dev)
    if n_local:
        payload = np.frombuffer(b"".join(local), np.uint8)
        buf[:payload.size] = torch.from_numpy(payload.copy()).to(dev)
    # payloads go to rank 0 only (a gather, not an all_gather: the other
    # ranks never need them)
    all_buf = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gather_list=all_buf, dst=0)
    if rank != 0:
        return None
    if not to_host:
        return all_buf, all_sz
    out = []
    for r in range(world):
        n = int(all_sz[r][0])
        lens = [int(x) for x in all_sz[r][1:n + 1]]
        data = all_buf[r].cpu().numpy().tobytes()
        off, lst = 0, []
        for L in lens:
            lst.append(data[off:off + L])
            off += L
        out.append(lst)
    return out


def scatter_streams(per_rank, dist, device=None):
    """The decode side of gather_streams: rank 0 holds one list of byte
    streams per rank (`per_rank`, ignored elsewhere); every rank gets its own
    list.  A broadcast of the padded sizes, then two scatters (sizes,
    payloads) -- RCCL over xGMI with "nccl", gloo on CPU."""
    import torch
    world = dist.get_world_size()
    rank = dist.get_rank()
    dev = device if device is not None else torch.device("cpu")
    head = torch.zeros(2, dtype=torch.int64, device=dev)
    if rank == 0:
        head[0] = max(len(x) for x in per_rank)
        head[1] = max(max(sum(len(s) for s in x) for x in per_rank), 1)
    dist.broadcast(head, src=0)
    maxn, maxb = int(head[0]), int(head[1])
    sz = torch.zeros(maxn + 1, dtype=torch.int64, device=dev)
    buf = torch.zeros(maxb, dtype=torch.uint8, device=dev)
    sz_list = buf_list = None
    if rank == 0:
        sz_list, buf_list = [], []
        for lst in per_rank:
            t = torch.zeros(maxn + 1, dtype=torch.int64)
            t[0] = len(lst)
            if lst:
                t[1:len(lst) + 1] = torch.tensor([len(x) for x in lst], dtype=torch.int64)
            b = torch.zeros(maxb, dtype=torch.uint8)
            if lst:
                payload = np.frombuffer(b"".join(lst), np.uint8)
                b[:payload.size] = torch.from_numpy(payload.copy())
            sz_list.append(t.to(dev))
            buf_list.append(b.to(dev))
    dist.scatter(sz, scatter_list=sz_list, src=0)
    dist.scatter(buf, scatter_list=buf_list, src=0)
    n = int(sz[0])
    data = buf.cpu().numpy().tobytes()
    out, off = [], 0
    for L in (int(x) for x in sz[1:n + 1]):
        out.append(data[off:off + L])
        off += L
    return out
