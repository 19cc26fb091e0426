"""Frame / tile sharding across GPUs and the gather of compressed .ric streams
(SURVEY.md §8(e)).

Independent frames (C3, C5) and tiles (C4) are independent .ric streams, so
ranks share no state while coding: frame f goes to rank f mod N, tile (tx, ty)
of a 2x2 grid to rank 2*ty + tx.  The only exchange is the gather of the
variable-size compressed streams to rank 0 (StreamGather): every stream a rank
codes, shipped in bounded chunks while the step still runs (a stream leaves as
soon as its .ric file is complete), so rank 0 holds at most one chunk per peer
whatever the step's size.  Transports: RCCL over xGMI between the GPUs
(RcclTransport: the library's own communicator, device buffers) and gloo on
the CPU (GlooTransport: the tests and the one-GPU rehearsals).

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


MAX_PER_CHUNK = 64          # streams per chunk (the header's capacity)
HDR_WORDS = 4 + 3 * MAX_PER_CHUNK
_DMUL = np.uint64(0x9E3779B97F4A7C15)


def digest_bytes(a):
    """The 64-bit digest of ric_batch_set_digests / ric_device_digests over a
    byte run: sum over byte k of a[k] * (k * 0x9E3779B97F4A7C15 + 1) mod 2^64."""
    a = np.frombuffer(a, np.uint8) if not isinstance(a, np.ndarray) else a.reshape(-1)
    if a.size == 0:
        return np.uint64(0)
    v = a.astype(np.uint64)
    with np.errstate(over="ignore"):
        s1 = np.uint64(np.sum(v, dtype=np.uint64))
        s2 = np.uint64(np.dot(v, np.arange(a.size, dtype=np.uint64)))
        return np.uint64(s2 * _DMUL + s1)


def _host_digests(buf, offs, lens):
    """Digests of host byte runs: the library's native loop (ric_host_digests,
    no GPU needed) when it loads, else numpy."""
    try:
        import ric_amd
        return ric_amd.host_digests(buf, offs, lens)
    except (ImportError, OSError):
        return np.array([digest_bytes(buf[o:o + n]) for o, n in zip(offs, lens)], np.uint64)


def _as_u8(data):
    return np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray) else data.reshape(-1)


class GlooTransport:
    """The gather's CPU transport: torch.distributed (gloo) point-to-point on
    host buffers (numpy uint8 arrays)."""

    def __init__(self, dist):
        self.dist = dist

    def alloc(self, nbytes):
        return np.zeros(max(int(nbytes), 16), np.uint8)

    def put(self, buf, off, data):
        src = _as_u8(data)
        buf[off:off + src.size] = src

    def put_many(self, buf, srcs, offs):
        """Streams into buf at offs (the gaps zeroed); returns their digests."""
        at = 0
        for x, o in zip(srcs, offs):
            x = _as_u8(x)
            if o > at:
                buf[at:o] = 0
            buf[o:o + x.size] = x
            at = o + x.size
        return _host_digests(buf, offs, [_as_u8(x).size for x in srcs])

    def get(self, buf, off, n):
        return buf[off:off + n]

    def sendrecv(self, ops):
        import torch
        reqs = []
        for peer, is_send, buf, n in ops:
            if not n:
                continue
            t = torch.from_numpy(buf[:n])
            reqs.append(self.dist.isend(t, peer) if is_send else self.dist.irecv(t, peer))
        for r in reqs:
            r.wait()

    def digests(self, buf, offs, lens):
        return _host_digests(buf, offs, lens)


class RcclTransport:
    """The gather's GPU transport: the library's RCCL communicator (ric_comm,
    xGMI between the GPUs of a node) on device buffers.  A chunk's streams go
    from their host buffers to the device in one copy through the library's
    pinned staging (ric_device_pack_h2d, digests taken on the way); rank 0
    digests what it received on the device (ric_device_digests).  Every copy
    and digest runs on the library's side stream and RCCL on the
    communicator's: none waits for the stream coder's kernel in flight."""

    def __init__(self, comm, device=0):
        import ric_amd
        self.R = ric_amd
        self.comm = comm
        self.device = device
        self._pinned = None

    def alloc(self, nbytes):
        return self.R.DeviceArray(max(int(nbytes), 16), np.uint8, self.device)

    def put(self, buf, off, data):
        src = _as_u8(data)
        if src.size:
            self.R._chk(self.R.lib().ric_device_copy(self.device, buf.data_ptr() + off, src.ctypes.data, src.size,
                                                     self.R.RIC_COPY_H2D), "gather H2D")

    def put_many(self, buf, srcs, offs):
        return self.R.device_pack_h2d(self.device, buf, srcs, offs)

    def get(self, buf, off, n):
        # into one pinned sink buffer, reused every round (rank 0 holds no more)
        if self._pinned is None or self._pinned.size < n:
            self._pinned = self.R.pinned_array(max(n, 1 << 20))
        if n:
            self.R._chk(self.R.lib().ric_device_copy(self.device, self._pinned.ctypes.data, buf.data_ptr() + off, n,
                                                     self.R.RIC_COPY_D2H), "gather D2H")
        return self._pinned[:n]

    def sendrecv(self, ops):
        self.comm.sendrecv([(p, s, b, n) for p, s, b, n in ops if n])

    def digests(self, buf, offs, lens):
        return self.R.device_digests(self.device, buf.data_ptr(), list(offs), list(lens))


class StreamGather:
    """The gather of every rank's .ric streams to rank 0, in bounded chunks.

    A round: every sender still active sends one chunk -- a header (round,
    count, done, payload bytes, then per stream: its index, length and
    digest) and the payload (whole streams back to back at 16-byte offsets,
    at most `chunk_bytes`, at most MAX_PER_CHUNK streams), as two point-to-point operations -- and
    rank 0 receives the headers, then the payloads, checks each stream's
    digest against the sender's, and hands each stream to
    `on_stream(rank, index, bytes)` from its sink buffer.  A sender takes into
    a chunk the streams that are ready (any order) and waits only when none
    is; its last chunk carries `done`.  Rank 0's memory: one chunk buffer per
    peer on the transport, whatever the number of streams; a peer whose chunk
    is larger (its header announces the payload's size) grows that buffer.
    """

    def __init__(self, transport, rank, world, chunk_bytes=64 << 20, max_chunk=1 << 30):
        self.t = transport
        self.rank, self.world = rank, world
        self.chunk = int(chunk_bytes)
        # the largest chunk a peer's header may announce (rank 0 grows that
        # peer's buffer to it; a corrupt header cannot ask for more)
        self.max_chunk = max(int(max_chunk), self.chunk)
        self.hdr = [self.t.alloc(HDR_WORDS * 8) for _ in range(max(world - 1, 1))]
        if rank == 0:
            self.bufs = [self.t.alloc(self.chunk) for _ in range(world - 1)]
            self.cap = [self.chunk] * max(world - 1, 1)
        else:
            self.bufs = [self.t.alloc(self.chunk)]
            self.cap = [self.chunk]
        self.stats = {}

    # ---- sender
    def send(self, n, words, data, poll_s=0.0005, stop=None, bias=0):
        """Ship streams 0..n-1 of this rank.  words: a uint32 array whose
        word i becomes stream i's length + bias once it is ready
        (ric_batch_set_ready: bias 0, every .ric file is at least 9 bytes;
        0 until then); data(i, length) -> its bytes (host).  stop(): an
        optional check that raises when the producer failed."""
        import time
        pending = np.ones(n, bool)
        left = n
        rnd = sent = nbytes = 0
        hdr = np.zeros(HDR_WORDS, np.int64)
        while True:
            take, offs, off = [], [], 0
            while True:
                cand = np.flatnonzero(pending & (words[:n] != 0)) if left else []
                for i in cand[:MAX_PER_CHUNK]:
                    ln = int(words[i]) - bias
                    if ln > self.chunk:
                        raise ValueError("stream %d (%d bytes) larger than the gather chunk (%d)" % (i, ln, self.chunk))
                    o = (off + 15) & ~15
                    if o + ln > self.chunk:
                        break
                    take.append((int(i), ln))
                    offs.append(o)
                    off = o + ln
                if take or not left:
                    break
                if stop is not None:
                    stop()
                time.sleep(poll_s)
            for i, _ in take:
                pending[i] = False
            left -= len(take)
            dg = np.asarray(self.t.put_many(self.bufs[0], [data(i, ln) for i, ln in take], offs), np.uint64)
            hdr[:] = 0
            hdr[0], hdr[1], hdr[2], hdr[3] = rnd, len(take), int(left == 0), off
            for k, (i, ln) in enumerate(take):
                hdr[4 + 3 * k], hdr[5 + 3 * k] = i, ln
            hdr[6:6 + 3 * len(take):3] = dg.view(np.int64)
            self.t.put(self.hdr[0], 0, hdr.view(np.uint8))
            # header and payload as two operations, as rank 0 receives them (it
            # reads the header on the host in between): the same grouping on
            # both sides of every RCCL transfer
            self.t.sendrecv([(0, True, self.hdr[0], HDR_WORDS * 8)])
            self.t.sendrecv([(0, True, self.bufs[0], off)])
            sent += len(take)
            nbytes += off
            rnd += 1
            if not left:
                break
        self.stats = {"rounds": rnd, "streams": sent, "bytes": nbytes}
        return self.stats

    # ---- rank 0
    def receive(self, on_stream=None, to_host=True):
        """Receive every peer's streams; returns per-rank counts and bytes and
        the digest mismatches.  to_host: every chunk also lands in the
        transport's host sink (where a server would write the files out)."""
        import time
        active = list(range(1, self.world))
        counts = [0] * self.world
        nbytes = [0] * self.world
        bad = []
        rnd = 0
        t_busy = 0.0
        while active:
            self.t.sendrecv([(r, False, self.hdr[r - 1], HDR_WORDS * 8) for r in active])
            t0 = time.perf_counter()
            heads = {}
            for r in active:
                h = np.frombuffer(bytes(self.t.get(self.hdr[r - 1], 0, HDR_WORDS * 8)), np.int64).copy()
                if h[0] != rnd or h[1] > MAX_PER_CHUNK or h[3] < 0 or h[3] > self.max_chunk:
                    raise RuntimeError("gather: bad chunk header from rank %d (round %d): %s" % (r, rnd, h[:4]))
                if h[3] > self.cap[r - 1]:
                    # a peer with a larger chunk (e.g. gather_streams' per-rank sizes)
                    self.bufs[r - 1] = self.t.alloc(int(h[3]))
                    self.cap[r - 1] = int(h[3])
                heads[r] = h
            self.t.sendrecv([(r, False, self.bufs[r - 1], int(heads[r][3])) for r in active])
            for r in active:
                h = heads[r]
                k = int(h[1])
                idx = h[4:4 + 3 * k:3]
                ln = h[5:5 + 3 * k:3]
                want = h[6:6 + 3 * k:3].view(np.uint64)
                offs, o = [], 0
                for L in ln:
                    o = (o + 15) & ~15
                    offs.append(o)
                    o += int(L)
                got = self.t.digests(self.bufs[r - 1], offs, [int(L) for L in ln])
                for j in range(k):
                    if got[j] != want[j]:
                        bad.append((r, int(idx[j])))
                if k and (on_stream is not None or to_host):
                    sink = self.t.get(self.bufs[r - 1], 0, int(h[3]))
                    if on_stream is not None:
                        for j in range(k):
                            on_stream(r, int(idx[j]), sink[offs[j]:offs[j] + int(ln[j])])
                counts[r] += k
                nbytes[r] += int(h[3])
            t_busy += time.perf_counter() - t0
            active = [r for r in active if not heads[r][2]]
            rnd += 1
        self.stats = {"rounds": rnd, "streams": counts, "bytes": nbytes, "digest_mismatches": bad,
                      "rank0_busy_s": t_busy}
        return self.stats


def gather_streams(local, transport, rank, world, chunk_bytes=1 << 20):
    """One-shot gather of byte streams (e.g. C4's tiles): rank 0 gets every
    rank's list in rank order (its own first), others None.  Each sender's
    chunk fits its own longest stream; rank 0 grows a peer's buffer to what
    that peer's header announces.  Empty streams are shipped too."""
    g = StreamGather(transport, rank, world, max(chunk_bytes, max([len(s) for s in local] + [16]) + 16))
    if rank != 0:
        g.send(len(local), np.array([len(x) + 1 for x in local], np.uint32), lambda i, n: local[i], bias=1)
        return None
    got = [dict() for _ in range(world)]
    g.receive(lambda r, i, b: got[r].__setitem__(i, bytes(b)))
    if g.stats["digest_mismatches"]:
        raise RuntimeError("gather: digest mismatches %s" % g.stats["digest_mismatches"][:8])
    return [list(local)] + [[got[r][i] for i in sorted(got[r])] for r in range(1, world)]


def scatter_streams(per_rank, transport, rank, world):
    """The decode side of gather_streams: rank 0 holds one list of byte
    streams per rank (`per_rank`, ignored elsewhere); every rank gets its own
    list.  Per peer: a count, the lengths, then the payload, point to point."""
    if rank == 0:
        for r in range(1, world):
            lst = per_rank[r]
            cnt = np.array([len(lst)], np.int64)
            lens = np.array([len(x) for x in lst] or [0], np.int64)
            payload = b"".join(lst)
            cb = transport.alloc(8)
            transport.put(cb, 0, cnt.view(np.uint8))
            lb = transport.alloc(lens.nbytes)
            transport.put(lb, 0, lens.view(np.uint8))
            pb = transport.alloc(len(payload))
            transport.put(pb, 0, payload)
            # one operation per message, as the peer receives them
            transport.sendrecv([(r, True, cb, 8)])
            transport.sendrecv([(r, True, lb, 8 * len(lst))])
            transport.sendrecv([(r, True, pb, len(payload))])
        return list(per_rank[0])
    cb = transport.alloc(8)
    transport.sendrecv([(0, False, cb, 8)])
    k = int(np.frombuffer(bytes(transport.get(cb, 0, 8)), np.int64)[0])
    lb = transport.alloc(8 * max(k, 1))
    transport.sendrecv([(0, False, lb, 8 * k)])
    lens = [int(x) for x in np.frombuffer(bytes(transport.get(lb, 0, 8 * k)), np.int64)] if k else []
    pb = transport.alloc(sum(lens))
    transport.sendrecv([(0, False, pb, sum(lens))])
    data = bytes(transport.get(pb, 0, sum(lens)))
    out, off = [], 0
    for L in lens:
        out.append(data[off:off + L])
        off += L
    return out
