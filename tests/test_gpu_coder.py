"""The serial .ric coder on the GPU (gcoder.hip: one wave per frame's stream)
against the oracle and the golden vectors: ric_batch_encode_gpu must write the
same .ric bytes as the reference's CompressImage."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def _slots(n, c):
    return n if c == 1 else (3 * n + 1) // 2          # colour: three plane pyramids per frame in 2 x slots arenas


def _gpu_encode(ric, frames, q, t):
    c, h, w = frames[0].shape[-3:]
    dev = [ric.DeviceArray.from_numpy(f) for f in frames]
    b = ric.Batch(w, h, c, slots=_slots(len(frames), c), threads=1)
    ostride = (w * h * c * 2 + 65536 + 4095) // 4096 * 4096
    out = ric.DeviceArray(len(frames) * ostride, np.uint8, zero=True)
    lens = b.compress_gpu(dev, out, ostride, q, t)
    host = out.numpy()
    return [host[i * ostride:i * ostride + n].tobytes() for i, n in enumerate(lens)]


@pytest.mark.parametrize("w,h,q,t", [(1024, 768, 9, 0), (640, 480, 0, 1), (328, 200, 20, 0), (257, 129, 9, 0),
                                     (128, 96, 9, 2), (1001, 603, 0, 1), (33, 47, 9, 0), (17, 16, 0, 1),
                                     (100, 60, 31, 0), (129, 77, 1, 1), (520, 392, 5, 0)])
def test_gpu_coder_matches_oracle(ric, port, w, h, q, t):
    frames = [ric.synth(w, h, 1, 60 + i) for i in range(3)]
    got = _gpu_encode(ric, frames, q, t)
    for f, r in zip(frames, got):
        assert r == port.encode_ric(f, q, t)


def test_gpu_coder_golden_small(ric):
    """Every small gray golden .ric of the reference, re-encoded on the GPU."""
    n = 0
    for e in G["small"]:
        if e["channels"] != 1:
            continue
        frame = ric.synth(e["w"], e["h"], 1, e["frame"])
        got = _gpu_encode(ric, [frame], e["q"], e["trans"])[0]
        assert got == open(os.path.join(HERE, "golden", e["name"] + ".ric"), "rb").read(), e["name"]
        n += 1
    assert n >= 8


@pytest.mark.parametrize("name", ["C3_7680x4320_q9", "C2_4096x4096_q9"])
def test_gpu_coder_large_sha(ric, name):
    """Full-size frames: the reference's own SHA-256 of the .ric file."""
    e = [x for x in G["large"] if x["name"] == name][0]
    w, h = e["w"], e["h"]
    frame = ric.synth(w, h, 1, e["frame"])
    got = _gpu_encode(ric, [frame], e["q"], e["trans"])[0]
    assert hashlib.sha256(got).hexdigest() == e["ric_sha256"]


@pytest.mark.parametrize("gpu_decode", [0, 1, 2])
@pytest.mark.parametrize("w,h,q,t,n,n_host,pool,slots", [(640, 480, 9, 0, 11, 3, 4, 3), (328, 200, 20, 0, 7, 0, 3, 2),
                                                         (257, 129, 9, 0, 5, 5, 2, 2), (1024, 768, 9, 0, 9, 2, 8, 4),
                                                         (128, 96, 0, 1, 6, 1, 2, 4), (96, 80, 9, 2, 7, 0, 2, 2)])
def test_hybrid_roundtrip(ric, port, w, h, q, t, n, n_host, pool, slots, gpu_decode):
    """GPU-encoded and host-encoded frames in one pipelined call (several
    coder launches, both halves of the stream buffer, both slot sets)."""
    host = [ric.synth(w, h, 1, 80 + i) for i in range(n)]
    frames = [ric.DeviceArray.from_numpy(x) for x in host]
    outs = [f.empty_like() for f in frames]
    b = ric.Batch(w, h, 1, slots=slots, threads=3)
    b.hybrid_config(pool, (w * h * 2 + 65536 + 15) // 16 * 16)
    for rep in range(2):
        lens = b.roundtrip_hybrid(frames, outs, n_host, q, t, gpu_decode=gpu_decode)
        for i in range(n):
            r = b.stream(i)
            assert len(r) == lens[i]
            assert r == port.encode_ric(host[i], q, t), (rep, i)
            assert np.array_equal(outs[i].numpy(), port.decode_ric(r)[0]), (rep, i)


def _pixel_digest(pix):
    flat = np.ascontiguousarray(pix, np.uint8).reshape(-1).astype(np.uint64)
    mult = np.arange(flat.size, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1)
    return np.uint64(np.sum(flat * mult, dtype=np.uint64))


@pytest.mark.parametrize("w,h,q", [(640, 360, 9), (1004, 600, 9), (333, 201, 9), (512, 256, 0)])
def test_hybrid_digests_and_fused_pixels(ric, port, w, h, q):
    """The serving step's pixel output fused into the inverse level 0 of gray
    9/7 frames (ZFrames::pix; widths a multiple of 4; others, e.g. 333, take
    the separate pixel kernel): every frame's pixels and its digest
    (ric_batch_set_digests, 16 partial words folded per frame) equal the
    oracle's, for host-coded and GPU-coded frames, with and without the
    fusion (RIC_PIX_FUSE is read once per process: the unfused form is the
    odd width here)."""
    n, n_host = 9, 3
    host = [ric.synth(w, h, 1, 140 + i) for i in range(n)]
    frames = [ric.DeviceArray.from_numpy(x) for x in host]
    outs = [f.empty_like() for f in frames]
    dig = ric.DeviceArray(n, np.uint64, zero=True)
    b = ric.Batch(w, h, 1, slots=3, threads=3)
    b.set_digests(dig, n)
    b.hybrid_config(3, (w * h * 2 + 65536 + 15) // 16 * 16)
    b.roundtrip_hybrid(frames, outs, n_host, q, 0, gpu_decode=1)
    got = dig.numpy()
    for i in range(n):
        r = b.stream(i)
        assert r == port.encode_ric(host[i], q, 0), i
        want = port.decode_ric(r)[0]
        assert np.array_equal(outs[i].numpy().reshape(want.shape), want), i
        assert got[i] == _pixel_digest(want), i


def _gpu_decode(ric, rics, w, h, c=1):
    istride = (max(len(r) for r in rics) + 4095) // 4096 * 4096
    buf = np.zeros(len(rics) * istride, np.uint8)
    for i, r in enumerate(rics):
        buf[i * istride:i * istride + len(r)] = np.frombuffer(r, np.uint8)
    src = ric.DeviceArray.from_numpy(buf)
    outs = [ric.DeviceArray((c, h, w), np.uint8, zero=True) for _ in rics]
    b = ric.Batch(w, h, c, slots=_slots(len(rics), c), threads=1)
    rc = b.decompress_gpu(src, istride, [len(r) for r in rics], outs)
    return rc, [o.numpy() for o in outs]


@pytest.mark.parametrize("w,h,q,t", [(1024, 768, 9, 0), (640, 480, 0, 1), (328, 200, 20, 0), (257, 129, 9, 0),
                                     (128, 96, 9, 2), (33, 47, 9, 0), (17, 16, 0, 1), (100, 60, 31, 0),
                                     (129, 77, 1, 1), (520, 392, 5, 0)])
def test_gpu_decoder_matches_oracle(ric, port, w, h, q, t):
    frames = [ric.synth(w, h, 1, 90 + i) for i in range(3)]
    rics = [port.encode_ric(f, q, t) for f in frames]
    rc, got = _gpu_decode(ric, rics, w, h)
    for r, g in zip(rics, got):
        assert np.array_equal(g.reshape(h, w), port.decode_ric(r)[0].reshape(h, w))


def test_gpu_decoder_desync_streams(ric, port):
    """1001x603 lossless: the reference's maxCode(v, 0) leaves its own decoder
    desynchronised; what it decodes after that is undefined
    behaviour (its models indexed out of range), pinned by the golden frame 0
    only.  The GPU decoder must decode exactly what the product's host decoder
    decodes, frame for frame."""
    w, h = 1001, 603
    rics = [port.encode_ric(ric.synth(w, h, 1, 90 + i), 0, 1) for i in range(3)]
    rc, got = _gpu_decode(ric, rics, w, h)
    b = ric.Batch(w, h, 1, slots=3, threads=2)
    for g, want in zip(got, b.decompress(rics)):
        assert np.array_equal(g.reshape(h, w), want.reshape(h, w))


def test_gpu_decoder_golden_small(ric):
    n = 0
    for e in G["small"]:
        if e["channels"] != 1:
            continue
        r = open(os.path.join(HERE, "golden", e["name"] + ".ric"), "rb").read()
        rc, got = _gpu_decode(ric, [r], e["w"], e["h"])
        assert hashlib.sha256(got[0].tobytes()).hexdigest() == e["decoded_sha256"], e["name"]
        n += 1
    assert n >= 8


@pytest.mark.parametrize("name", ["C3_7680x4320_q9", "C2_4096x4096_q9", "lossless53_1001x603"])
def test_gpu_roundtrip_large_sha(ric, name):
    """Encode and decode on the GPU: the reference's SHA-256 of both."""
    e = [x for x in G["large"] if x["name"] == name][0]
    w, h = e["w"], e["h"]
    frame = ric.DeviceArray.from_numpy(ric.synth(w, h, 1, e["frame"]))
    b = ric.Batch(w, h, 1, slots=1, threads=1)
    ostride = (w * h * 2 + 65536 + 4095) // 4096 * 4096
    out = ric.DeviceArray(ostride, np.uint8, zero=True)
    lens = b.compress_gpu([frame], out, ostride, e["q"], e["trans"])
    assert hashlib.sha256(out.numpy()[:lens[0]].tobytes()).hexdigest() == e["ric_sha256"]
    pix = ric.DeviceArray((1, h, w), np.uint8, zero=True)
    b.decompress_gpu(out, ostride, lens, [pix])
    assert hashlib.sha256(pix.numpy().tobytes()).hexdigest() == e["decoded_sha256"]


def test_gpu_encoder_rejects_unaligned_capacity(ric):
    """The stream coder stores 16-byte chunks: a capacity or stride that is not
    a multiple of 16 would drop a stream's tail unflagged, so it is refused."""
    import ctypes
    w, h = 64, 48
    frame = ric.DeviceArray.from_numpy(ric.synth(w, h, 1, 1))
    b = ric.Batch(w, h, 1, slots=1, threads=1)
    out = ric.DeviceArray(65536, np.uint8, zero=True)
    lens = (ctypes.c_size_t * 1)()
    for ostride, cap in ((8192, 8190), (8200, 8192), (8192, 8192)):
        rc = ric.lib().ric_batch_encode_gpu(b.h, ric._ptrs([frame]), 1, 9, 0, out.data_ptr(), ostride, cap, lens)
        assert rc == (ric.RIC_OK if (cap, ostride) == (8192, 8192) else ric.RIC_E_ARG), (ostride, cap)


@pytest.mark.parametrize("w,h,q,t", [(320, 240, 9, 0), (129, 77, 5, 0), (640, 480, 0, 1), (257, 129, 20, 0)])
def test_gpu_coder_colour_matches_oracle(ric, port, w, h, q, t):
    """RGB: Y, Co, Cg coded one after the other into one stream on one wave
    (ric.cpp:157-176, chroma quantisers +C_Q_BOOST), both directions"""
    frames = [ric.synth(w, h, 3, 70 + i) for i in range(3)]
    got = _gpu_encode(ric, frames, q, t)
    for f, r in zip(frames, got):
        assert r == port.encode_ric(f, q, t)
    rc, dec = _gpu_decode(ric, got, w, h, 3)
    for r, g in zip(got, dec):
        assert np.array_equal(g.reshape(-1), port.decode_ric(r)[0].reshape(-1))


def test_gpu_coder_colour_golden_small(ric):
    n = 0
    for e in G["small"]:
        if e["channels"] != 3:
            continue
        frame = ric.synth(e["w"], e["h"], 3, e["frame"])
        gold = open(os.path.join(HERE, "golden", e["name"] + ".ric"), "rb").read()
        assert _gpu_encode(ric, [frame], e["q"], e["trans"])[0] == gold, e["name"]
        rc, got = _gpu_decode(ric, [gold], e["w"], e["h"], 3)
        assert hashlib.sha256(got[0].tobytes()).hexdigest() == e["decoded_sha256"], e["name"]
        n += 1
    assert n >= 1


def test_gpu_coder_colour_large_sha(ric):
    """8K RGB through the GPU stream coder both ways: the reference's SHA-256"""
    e = [x for x in G["large"] if x["name"] == "C3rgb_7680x4320_q9"][0]
    w, h = e["w"], e["h"]
    got = _gpu_encode(ric, [ric.synth(w, h, 3, e["frame"])], e["q"], e["trans"])[0]
    assert hashlib.sha256(got).hexdigest() == e["ric_sha256"]
    rc, dec = _gpu_decode(ric, [got], w, h, 3)
    assert hashlib.sha256(dec[0].tobytes()).hexdigest() == e["decoded_sha256"]


def test_hybrid_tagged_results_across_launch_forms(ric, port):
    """Repeated calls on one batch alternate the merged k_gc_roundtrip launch
    over both pool halves, per-half k_gc_encode launches (a call with one
    coder batch, a call's third batch, lossless streams), odd pool and slot
    geometries, and new frames every call: each stream copier must take only
    its own launch's posted results (tagged per launch), never a word an
    earlier launch left over the same frames.  The stream-ready words
    (ric_batch_set_ready) carry every frame's length."""
    w, h = 200, 136
    b = ric.Batch(w, h, 1, slots=3, threads=2)
    b.hybrid_config(5, (w * h * 2 + 65536 + 15) // 16 * 16)
    plan = [(13, 2, 9, 0), (4, 0, 9, 0), (13, 1, 20, 0), (11, 0, 0, 1), (9, 3, 9, 0), (3, 3, 9, 0), (12, 1, 5, 0),
            (12, 1, 5, 0)]
    for call, (n, n_host, q, t) in enumerate(plan):
        host = [ric.synth(w, h, 1, 300 + 17 * call + i) for i in range(n)]
        frames = [ric.DeviceArray.from_numpy(x) for x in host]
        outs = [f.empty_like() for f in frames]
        words = np.zeros(n, np.uint32)
        b.set_ready(words, n)
        lens = b.roundtrip_hybrid(frames, outs, n_host, q, t, gpu_decode=1)
        b.set_ready(None, 0)
        assert list(words) == lens, call
        for i in range(n):
            r = b.stream(i)
            assert r == port.encode_ric(host[i], q, t), (call, i)
            assert np.array_equal(outs[i].numpy(), port.decode_ric(r)[0]), (call, i)


def test_device_digests_and_comm_self(ric):
    """The gather's device primitives: ric_device_digests = shard.digest_bytes
    (the host formula); a one-rank RCCL communicator sending to itself; the
    all-reduce; a StreamGather-style chunk through RcclTransport."""
    import shard
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    d = ric.DeviceArray.from_numpy(data)
    offs, lens = [0, 16, 1000, 4099, 65536], [1, 999, 3000, 70000, 900000]
    got = ric.device_digests(0, d, offs, lens)
    for o, n, g in zip(offs, lens, got):
        assert g == shard.digest_bytes(data[o:o + n]), (o, n)
    comm = ric.Comm(ric.Comm.unique_id(), 1, 0, 0)
    assert comm.allreduce([3.0, -1.5], ric.RIC_RED_SUM).tolist() == [3.0, -1.5]
    back = ric.DeviceArray(data.size, np.uint8, zero=True)
    comm.sendrecv([(0, True, d, data.size), (0, False, back, data.size)])
    assert np.array_equal(back.numpy(), data)
    t = shard.RcclTransport(comm, 0)
    buf = t.alloc(1 << 16)
    t.put(buf, 32, data[:5000])
    assert bytes(t.get(buf, 32, 5000)) == data[:5000].tobytes()
    assert t.digests(buf, [32], [5000])[0] == shard.digest_bytes(data[:5000])


@pytest.mark.parametrize("gpu_decode", [1, 0, 2])
@pytest.mark.parametrize("w,h,q,t,n,n_host,pool,slots", [(256, 192, 9, 0, 8, 2, 3, 6), (129, 77, 5, 0, 7, 1, 2, 4),
                                                         (160, 96, 0, 1, 5, 2, 2, 3)])
def test_hybrid_roundtrip_colour(ric, port, w, h, q, t, n, n_host, pool, slots, gpu_decode):
    """RGB frames through the serving step: the GPU stream coder codes each
    frame's Y, Co, Cg pyramids into one stream on one wave (ric.cpp:157-176);
    host round trips beside it keep each plane in a slot of its own."""
    host = [ric.synth(w, h, 3, 120 + i) for i in range(n)]
    frames = [ric.DeviceArray.from_numpy(x) for x in host]
    outs = [f.empty_like() for f in frames]
    b = ric.Batch(w, h, 3, slots=slots, threads=3)
    b.hybrid_config(pool, (w * h * 3 * 2 + 65536 + 15) // 16 * 16)
    for rep in range(2):
        b.roundtrip_hybrid(frames, outs, n_host, q, t, gpu_decode=gpu_decode)
        for i in range(n):
            r = b.stream(i)
            assert r == port.encode_ric(host[i], q, t), (rep, i)
            assert np.array_equal(outs[i].numpy(), port.decode_ric(r)[0].reshape(3, h, w)), (rep, i)


@pytest.mark.parametrize("gpu_decode,c", [(1, 1), (0, 1), (1, 3)])
def test_hybrid_compacted_pool_capacity(ric, port, gpu_decode, c):
    """The compacted pool (ric_batch_hybrid_config_ex): level 0 held as its
    non-zero values + block masks, the encoder reading and the decoder writing
    that form, the harvest expanding it.  The default capacity, the dense pool
    (0) and a capacity the synthetic frames exceed (flat frames fit, so one call
    mixes both): a frame over the capacity is coded on the host instead, with
    the same bytes, ready word and pixel digest."""
    import shard
    w, h, n = 256, 192, 7
    host = [np.full((c, h, w), 100 + i, np.uint8) if i % 2 else ric.synth(w, h, c, 400 + i) for i in range(n)]
    frames = [ric.DeviceArray.from_numpy(x) for x in host]
    want = [port.encode_ric(x, 9, 0) for x in host]
    for vc in (-1, 0, 200):
        b = ric.Batch(w, h, c, slots=3, threads=2)
        b.hybrid_config(3, (w * h * c * 2 + 65536 + 15) // 16 * 16, vc)
        outs = [f.empty_like() for f in frames]
        words = np.zeros(n, np.uint32)
        dig = ric.DeviceArray(n, np.uint64, zero=True)
        b.set_ready(words, n)
        b.set_digests(dig, n)
        lens = b.roundtrip_hybrid(frames, outs, 1, 9, 0, gpu_decode=gpu_decode)
        b.set_ready(None, 0)
        b.set_digests(None, 0)
        assert list(words) == lens, vc
        d = dig.numpy()
        for i in range(n):
            assert b.stream(i) == want[i], (vc, i)
            px = outs[i].numpy()
            assert np.array_equal(px.reshape(-1), port.decode_ric(want[i])[0].reshape(-1)), (vc, i)
            assert d[i] == shard.digest_bytes(px), (vc, i)


@pytest.mark.parametrize("c,slots", [(1, 4), (3, 6)])
def test_hybrid_capacity_fallback_groups(ric, port, c, slots):
    """Every stream-coder frame over the compacted pool's capacity (consecutive
    frames): they go round trip on the host in groups of up to slots / c
    frames (round 5; one frame per group before), same bytes and pixels."""
    w, h, n = 192, 128, 10
    host = [ric.synth(w, h, c, 600 + i) for i in range(n)]
    frames = [ric.DeviceArray.from_numpy(x) for x in host]
    want = [port.encode_ric(x, 9, 0) for x in host]
    b = ric.Batch(w, h, c, slots=slots, threads=3)
    b.hybrid_config(4, (w * h * c * 2 + 65536 + 15) // 16 * 16, 64)
    outs = [f.empty_like() for f in frames]
    lens = b.roundtrip_hybrid(frames, outs, 1, 9, 0, gpu_decode=1)
    assert b.hybrid_fallbacks() == n - 1
    for i in range(n):
        assert lens[i] == len(want[i]) and b.stream(i) == want[i], i
        assert np.array_equal(outs[i].numpy().reshape(-1), port.decode_ric(want[i])[0].reshape(-1)), i


@pytest.mark.parametrize("slots", [1, 2])
def test_hybrid_colour_small_slots(ric, port, slots):
    """Colour frames need three slots per host-coded frame.  A compacted pool
    can leave any frame to a host round trip (over its value capacity), so a
    colour batch with fewer than three slots is refused up front when the pool
    is compacted, even with n_host 0 and GPU decode (it would index slots past
    the batch's arenas); the dense pool (value_cap 0) still runs it."""
    w, h, c, n = 128, 96, 3, 4
    host = [np.full((c, h, w), 90 + i, np.uint8) if i % 2 else ric.synth(w, h, c, 500 + i) for i in range(n)]
    frames = [ric.DeviceArray.from_numpy(x) for x in host]
    outs = [f.empty_like() for f in frames]
    b = ric.Batch(w, h, c, slots=slots, threads=2)
    b.hybrid_config(2, (w * h * c * 2 + 65536 + 15) // 16 * 16, 100)
    with pytest.raises(ric.RicError) as ei:
        b.roundtrip_hybrid(frames, outs, 0, 9, 0, gpu_decode=1)
    assert ei.value.rc == ric.RIC_E_ARG
    b.hybrid_config(2, (w * h * c * 2 + 65536 + 15) // 16 * 16, 0)
    b.roundtrip_hybrid(frames, outs, 0, 9, 0, gpu_decode=1)
    for i in range(n):
        r = b.stream(i)
        assert r == port.encode_ric(host[i], 9, 0), i
        assert np.array_equal(outs[i].numpy().reshape(-1), port.decode_ric(r)[0].reshape(-1)), i
