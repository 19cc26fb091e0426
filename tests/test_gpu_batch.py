"""ric_batch (the batched form of CompressImage / DecompressImage: one GPU
launch per level over a group of frames, a native host coder pool) against the
oracle and the golden vectors."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def large(name):
    return [e for e in G["large"] if e["name"] == name][0]


@pytest.mark.parametrize("w,h,ch,q,t", [(1024, 768, 1, 9, 0), (640, 480, 1, 0, 1), (328, 200, 1, 20, 0),
                                        (257, 129, 1, 9, 0), (256, 192, 3, 9, 0), (128, 96, 1, 9, 2),
                                        (96, 80, 3, 0, 1)])
def test_batch_encode_decode(ric, port, w, h, ch, q, t):
    frames = [ric.synth(w, h, ch, 20 + i) for i in range(5)]
    b = ric.Batch(w, h, ch, slots=5, threads=3)
    got = b.compress(frames, q, t)
    for f, r in zip(frames, got):
        assert r == port.encode_ric(f, q, t)
    dec = b.decompress(got)
    for r, d in zip(got, dec):
        assert np.array_equal(d, port.decode_ric(r)[0])
    # fewer frames than slots, then the full group again (argument arrays change size)
    assert b.compress(frames[:2], q, t) == got[:2]
    assert b.compress(frames, q, t) == got


def test_batch_mixed_q_decode(ric, port):
    """One decode call over streams of different q (per-frame TSUQi factors)."""
    w, h = 512, 384
    frames = [ric.synth(w, h, 1, i) for i in range(4)]
    rics = [port.encode_ric(f, q, 0) for f, q in zip(frames, [9, 3, 17, 9])]
    b = ric.Batch(w, h, 1, slots=4, threads=2)
    for r, d in zip(rics, b.decompress(rics)):
        assert np.array_equal(d, port.decode_ric(r)[0])


@pytest.mark.parametrize("slots,n", [(4, 11), (3, 3), (2, 5)])
def test_batch_roundtrip_pipeline(ric, port, slots, n):
    w, h = 768, 512
    host = [ric.synth(w, h, 1, 40 + i) for i in range(n)]
    frames = [ric.DeviceArray.from_numpy(x) for x in host]
    outs = [f.empty_like() for f in frames]
    b = ric.Batch(w, h, 1, slots=slots, threads=3)
    b.prof_enable(True)
    b.roundtrip(frames, outs, q=9, trans=0)
    for i in range(n):
        r = b.stream(i)
        assert r == port.encode_ric(host[i], 9, 0)
        assert np.array_equal(outs[i].numpy(), port.decode_ric(r)[0])
    prof = b.prof_read()
    assert prof["fwd_l0"][1] == n and prof["inv_l0"][1] == n and prof["host_enc"][1] == n


def test_batch_full_size_golden(ric):
    """C3 (8K) and C2/C5 (4096^2) frames through the batched pipeline against
    the reference's SHA-256 (frame 0 = C3 / C2, frame 1 = C5 frame 1)."""
    for (W, H, names) in [(7680, 4320, {0: "C3_7680x4320_q9"}),
                          (4096, 4096, {0: "C2_4096x4096_q9", 1: "C5_frame1_4096x4096_q9"})]:
        frames = [ric.DeviceArray.from_numpy(ric.synth(W, H, 1, f)) for f in range(3)]
        outs = [f.empty_like() for f in frames]
        b = ric.Batch(W, H, 1, slots=2, threads=3)
        b.roundtrip(frames, outs, q=9, trans=0)
        for f, nm in names.items():
            e = large(nm)
            r = b.stream(f)
            assert len(r) == e["ric_bytes"] and sha(r) == e["ric_sha256"], nm
            assert sha(outs[f].numpy().tobytes()) == e["decoded_sha256"], nm
        del b


def test_batch_c4_tiles(ric):
    """The four C4 tiles (3840x2160 RGB crops of the 8K RGB image) as one batch."""
    import shard
    rgb = ric.synth(7680, 4320, 3, 0)
    tiles, names = [], []
    for (tx, ty, x0, y0, w, h) in shard.tile_rects(7680, 4320):
        tiles.append(np.ascontiguousarray(rgb[:, y0:y0 + h, x0:x0 + w]))
        names.append("C4_tile_%d_%d" % (tx, ty))
    b = ric.Batch(3840, 2160, 3, slots=4, threads=4)
    got = b.compress(tiles, 9, 0)
    for r, nm in zip(got, names):
        assert sha(r) == large(nm)["ric_sha256"], nm
    for d, nm in zip(b.decompress(got), names):
        assert sha(d.tobytes()) == large(nm)["decoded_sha256"], nm


def test_batch_ring_timeout_is_an_error(ric, port):
    w, h = 1024, 768
    frames = [ric.synth(w, h, 1, i) for i in range(3)]
    b = ric.Batch(w, h, 1, slots=3, threads=2)
    lib = ric.lib()
    lib.ric_diag_fault(1)
    try:
        with pytest.raises(ric.RicError) as ei:
            b.compress(frames, 9, 0)
        assert ei.value.rc == ric.RIC_E_HIP and "ring" in str(ei.value)
    finally:
        lib.ric_diag_fault(0)
    got = b.compress(frames, 9, 0)
    assert got == [port.encode_ric(f, 9, 0) for f in frames]


def _digest(pix):
    flat = np.ascontiguousarray(pix, np.uint8).reshape(-1).astype(np.uint64)
    mult = np.arange(flat.size, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1)
    return np.uint64(np.sum(flat * mult, dtype=np.uint64))


@pytest.mark.parametrize("w,h,ch", [(768, 512, 1), (333, 201, 3)])
def test_batch_output_digests(ric, port, w, h, ch):
    """ric_batch_set_digests: every frame's digest is taken in stream order
    right after its pixels, so frames sharing one output buffer keep their own
    (the bench verifies its serving step this way)"""
    n = 7
    host = [ric.synth(w, h, ch, 50 + i) for i in range(n)]
    frames = [ric.DeviceArray.from_numpy(x) for x in host]
    shared = [frames[0].empty_like() for _ in range(2)]
    outs = [shared[i % 2] for i in range(n)]
    dig = ric.DeviceArray(n, np.uint64, zero=True)
    b = ric.Batch(w, h, ch, slots=2, threads=2)
    b.set_digests(dig, n)
    b.roundtrip(frames, outs, q=9, trans=0)
    got = dig.numpy()
    for i in range(n):
        want = port.decode_ric(port.encode_ric(host[i], 9, 0))[0]
        assert got[i] == _digest(want), i


@pytest.mark.parametrize("w,h,ch,q,t", [(1024, 768, 1, 9, 0), (640, 480, 1, 0, 1), (257, 129, 1, 9, 0),
                                        (256, 192, 3, 9, 0), (96, 80, 3, 0, 1)])
def test_batch_band_parallel_encode(ric, port, w, h, ch, q, t):
    """Fewer frames in flight than half the host threads (C4's tiles, C5 over
    many ranks): each frame's bands are modelled on the batch's band pool while
    its task writes the stream (encode_bands_split), over the compacted payload
    where the bands are 16-bit -- the same bytes as the oracle."""
    frames = [ric.synth(w, h, ch, 60 + i) for i in range(2)]
    b = ric.Batch(w, h, ch, slots=4, threads=8)
    for _ in range(2):
        got = b.compress(frames, q, t)
        for f, r in zip(frames, got):
            assert r == port.encode_ric(f, q, t)
    if ch == 1:
        dev = [ric.DeviceArray.from_numpy(f) for f in frames]
        outs = [d.empty_like() for d in dev]
        lens = b.roundtrip(dev, outs, q, t)
        for i, f in enumerate(frames):
            r = b.stream(i)
            assert len(r) == lens[i] and r == port.encode_ric(f, q, t)
            assert np.array_equal(outs[i].numpy(), port.decode_ric(r)[0])
