"""GPU path (through the C-ABI) against the golden vectors produced by the
reference library, at small and full sizes (BASELINE.json configs), plus the
drop-in API semantics (band dumps, explicit pyramid shapes)."""
import hashlib
import json
import os
import threading

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
G = json.load(open(os.path.join(GOLD, "golden.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def large(name):
    return [e for e in G["large"] if e["name"] == name][0]


@pytest.mark.parametrize("e", G["small"], ids=[e["name"] for e in G["small"]])
def test_small_golden(ric, e):
    pix = ric.synth(e["w"], e["h"], e["channels"], e["frame"])
    c = ric.Codec(e["w"], e["h"], e["channels"])
    gold = open(os.path.join(GOLD, e["name"] + ".ric"), "rb").read()
    assert c.compress(pix, e["q"], e["trans"]) == gold
    dec, planes = c.decompress(gold)
    assert sha(dec.tobytes()) == e["decoded_sha256"]
    assert sha(planes.astype("<i2").tobytes()) == e["planes_sha256"]


BAND_CASES = [(e, False) for e in G["bands"]] + [(e, True) for e in G["bands"] if e["stage"] == 1]


@pytest.mark.parametrize("e,fused", BAND_CASES, ids=[e["name"] + ("_fused" if f else "") for e, f in BAND_CASES])
def test_band_dumps_golden(ric, e, fused):
    """The reference's band dumps through the CWavelet2D mirror on the GPU:
    stage 0 Transform; stage 1 buildTree + LL TSUQ (Quantize, or the fused
    TransformQuantize); stage 2 the whole CodeBand (the bands the zerotree scan
    leaves, src/lib/bandcodec.cpp:510-588); stage 3 the closed loop CodeBand ->
    TSUQi -> TransformI (src/lib/rududucodec.cpp:67-74)."""
    w, h, t, st = e["w"], e["h"], e["trans"], e["stage"]
    pl = O.gray_plane(ric.synth(w, h, 1, 0)[0], e["q"])
    W = ric.Wavelet2D(w, h, e["levels"], e["lc"])
    W.SetWeight(t)
    if fused:
        W.TransformQuantize(pl, w, t, e["quant"], e["lambda"])
    else:
        W.Transform(pl, w, t)
    if st == 1 and not fused:
        W.Quantize(e["quant"], e["lambda"])
    if st >= 2:
        buf = np.zeros(w * h * 4 + 4096, np.uint8)
        m = ric.MuxCodec(buf, first_word=0)
        W.CodeBand(m, e["quant"], e["lambda"])
        m.endCoding()
    if st == 3:
        W.TSUQi(e["quant"] or 1)
        out = np.zeros((h, w), np.int16)
        W.TransformI(out, w, t)
        flat = out.ravel().astype(np.int32)
    else:
        flat = np.concatenate([b.ravel() for b in W.bands()])
    assert np.array_equal(flat, np.load(os.path.join(GOLD, e["name"] + ".npy")))


@pytest.mark.parametrize("w,h", [(300, 220), (129, 77), (640, 480)])
@pytest.mark.parametrize("t", [0, 1])
@pytest.mark.parametrize("L,lc", [(5, 1), (3, 0)])
def test_closed_loop(ric, port, w, h, t, L, lc):
    """CodeBand -> TSUQi -> TransformI through the C-ABI equals the oracle
    (bands after TSUQi and the reconstructed plane)."""
    pl = O.gray_plane(ric.synth(w, h, 1, 6)[0], 9)
    exp_plane, exp_bands = port.closed_loop(pl, L, lc, t, 96, 36, 96)
    W = ric.Wavelet2D(w, h, L, lc)
    W.SetWeight(t)
    W.Transform(pl, w, t)
    buf = np.zeros(w * h * 4 + 4096, np.uint8)
    m = ric.MuxCodec(buf, first_word=0)
    W.CodeBand(m, 96, 36)
    m.endCoding()
    W.TSUQi(96)
    for a, b in zip(W.bands(), exp_bands):
        assert np.array_equal(a, b)
    out = np.zeros((h, w), np.int16)
    W.TransformI(out, w, t)
    assert np.array_equal(out, exp_plane)


@pytest.mark.parametrize("t", [0, 1])
@pytest.mark.parametrize("quant", [96, 7, 1])
def test_tsuqi(ric, port, t, quant):
    """CWavelet2D::TSUQi (src/lib/wavelet2d.cpp:248-268, CBand::TSUQi
    src/lib/band.h:94-107: v *= (C)(Quant / Weight), float32, at least 1) on
    the raw transform (the k_dequant kernel), restated in numpy."""
    w, h = 257, 130
    pl = O.gray_plane(ric.synth(w, h, 1, 2)[0], 9)
    W = ric.Wavelet2D(w, h, 5, 1)
    W.SetWeight(t)
    W.Transform(pl, w, t)
    raw = W.bands()
    W.TSUQi(quant)
    got = W.bands()
    for i in range(W.band_count()):
        _, _, isint, wt = W.band_info(i)
        q = quant if isint else int(np.int16(quant))
        q = int(np.float32(q) / np.float32(wt))
        q = q if isint else int(np.int16(q))
        q = q or 1
        v = raw[i].astype(np.int64) * q
        exp = v.astype(np.int32) if isint else v.astype(np.int16).astype(np.int32)
        assert np.array_equal(got[i], exp), i


def test_c1_api_planes(ric):
    """C1: 512x512 lossless 5/3, 3 levels, level_chg -1, through the
    CWavelet2D/CMuxCodec mirror (not the .ric wrapper)."""
    e = large("C1_512x512_lossless_53_L3_lc-1")
    img = ric.synth(512, 512, 1)[0]
    pl = (img.astype(np.int32) - 128).astype(np.int16)
    W = ric.Wavelet2D(512, 512, 3, -1)
    W.SetWeight(1)
    buf = np.zeros(512 * 512 * 2, np.uint8)
    m = ric.MuxCodec(buf, first_word=0)
    W.Transform(pl, 512, 1)
    W.CodeBand(m, 0, 0)
    n = m.endCoding()
    assert n == e["stream_bytes"] and sha(buf[:n].tobytes()) == e["stream_sha256"]
    D = ric.Wavelet2D(512, 512, 3, -1)
    D.SetWeight(1)
    dm = ric.MuxCodec(buf[:n].copy(), length=n)
    D.DecodeBand(dm)
    out = np.zeros((512, 512), np.int16)
    D.TransformI(out, 512, 1)
    assert np.array_equal(out, pl)


@pytest.mark.parametrize("name", ["C2_4096x4096_q9", "C5_frame1_4096x4096_q9", "C3_7680x4320_q9",
                                  "lossless53_1001x603", "C3rgb_7680x4320_q9"])
def test_full_size(ric, name):
    e = large(name)
    pix = ric.synth(e["w"], e["h"], e["channels"], e["frame"])
    c = ric.Codec(e["w"], e["h"], e["channels"])
    r = c.compress(pix, e["q"], e["trans"])
    assert len(r) == e["ric_bytes"] and sha(r) == e["ric_sha256"]
    dec, _ = c.decompress(r)
    assert sha(dec.tobytes()) == e["decoded_sha256"]


def test_c4_tiles(ric):
    import shard
    rgb = ric.synth(7680, 4320, 3, 0)
    c = ric.Codec(3840, 2160, 3)
    streams = []
    for (tx, ty, x0, y0, w, h) in shard.tile_rects(7680, 4320):
        e = large("C4_tile_%d_%d" % (tx, ty))
        tile = np.ascontiguousarray(rgb[:, y0:y0 + h, x0:x0 + w])
        r = c.compress(tile, 9, 0)
        assert sha(r) == e["ric_sha256"]
        dec, _ = c.decompress(r)
        assert sha(dec.tobytes()) == e["decoded_sha256"]
        streams.append(r)
    W, H, nx, ny, back = shard.unpack_tiles(shard.pack_tiles(7680, 4320, 2, 2, streams))
    assert back == streams


def desync_prone(w, h):
    """A finest D/H/V band with a 1x1 corner block: maxCode(v, 0) writes no bit
    but maxDecode(0) reads one (src/lib/muxcodec.cpp:516-534), so the
    reference's own decoder desynchronises (and may crash) on such streams."""
    dims = [((w + 1) >> 1, (h + 1) >> 1), (w >> 1, (h + 1) >> 1), ((w + 1) >> 1, h >> 1)]
    return any(dx % 4 == 1 and dy % 4 == 1 for dx, dy in dims)


@pytest.mark.parametrize("w,h", [(8, 8), (15, 9), (16, 16), (31, 17), (257, 129), (2048, 24), (130, 66)])
@pytest.mark.parametrize("q,t", [(0, 1), (9, 0), (17, 0)])
def test_edge_geometries(ric, port, w, h, q, t):
    pix = ric.synth(w, h, 1, w + h)
    c = ric.Codec(w, h, 1)
    r = c.compress(pix, q, t)
    assert r == port.encode_ric(pix, q, t)
    dec = c.decompress(r)[1]              # must not crash, even when desynchronised
    if not desync_prone(w, h):
        assert np.array_equal(dec, port.decode_ric(r)[1])


@pytest.mark.parametrize("L,lc", [(1, 0), (2, 0), (3, -1), (4, 2), (6, 1), (5, 3)])
@pytest.mark.parametrize("t", [0, 1])
def test_pyramid_shapes(ric, port, L, lc, t):
    w, h = 300, 220
    pl = O.gray_plane(ric.synth(w, h, 1, 4)[0], 9)
    W = ric.Wavelet2D(w, h, L, lc)
    W.SetWeight(t)
    W.Transform(pl, w, t)
    for a, b in zip(W.bands(), port.bands(pl, L, lc, t, 0)):
        assert np.array_equal(a, b)
    buf = np.zeros(w * h * 4, np.uint8)
    m = ric.MuxCodec(buf, first_word=0)
    W.CodeBand(m, 96, 36)
    n = m.endCoding()
    assert buf[:n].tobytes() == port.encode_planes(pl[None], L, lc, t, [96], [36])


def test_concurrent_codecs(ric, port):
    """One codec per host thread (the bench's layout) gives the same bytes."""
    w, h = 640, 480
    frames = [ric.synth(w, h, 1, f) for f in range(6)]
    exp = [port.encode_ric(f, 9, 0) for f in frames]
    got = [None] * 6
    codecs = [ric.Codec(w, h, 1) for _ in range(3)]

    def run(k):
        for i in range(k, 6, 3):
            r = codecs[k].compress(frames[i], 9, 0)
            dec, _ = codecs[k].decompress(r)
            got[i] = (r, dec)

    ths = [threading.Thread(target=run, args=(k,)) for k in range(3)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    for i in range(6):
        assert got[i][0] == exp[i]
        assert np.array_equal(got[i][1], port.decode_ric(exp[i])[0])


def test_device_resident_buffers(ric, port):
    w, h = 1024, 768
    pix = ric.synth(w, h, 1, 3)
    d = ric.DeviceArray.from_numpy(pix)
    out = d.empty_like()
    c = ric.Codec(w, h, 1)
    r = c.compress(d, 9, 0, on_device=True)
    assert r == port.encode_ric(pix, 9, 0)
    c.decompress(r, pix_out=out)
    ric.device_sync()
    assert np.array_equal(out.numpy(), port.decode_ric(r)[0])


@pytest.mark.parametrize("kind", ["uniform", "alt", "ramp"])
@pytest.mark.parametrize("w,h", [(64, 48), (96, 64), (129, 77), (256, 128)])
@pytest.mark.parametrize("t", [0, 1])
def test_full_range_planes(ric, port, kind, w, h, t):
    """Planes whose 9/7 lifting sums leave 16 bits (the video residual, any
    API caller): mult08 of a sum runs in int in the reference
    (src/lib/wavelet2d.cpp:336 deduces C = int), so every kernel takes the
    exact form (dwt.hip mult08x).  Forward (unfused k_fwd and the fused
    packed/generic kernels), buildTree and the closed loop's inverse."""
    pl = O.full_range_plane(w, h, w * h, kind)
    for L, lc in [(3, 0), (5, 1)]:
        W = ric.Wavelet2D(w, h, L, lc)
        W.SetWeight(t)
        W.Transform(pl, w, t)
        for a, b in zip(W.bands(), port.bands(pl, L, lc, t, 0)):
            assert np.array_equal(a, b), ("stage 0", L, lc)
        W = ric.Wavelet2D(w, h, L, lc)
        W.SetWeight(t)
        W.TransformQuantize(pl, w, t, 96, 36)
        for a, b in zip(W.bands(), port.bands(pl, L, lc, t, 1, 96, 36)):
            assert np.array_equal(a, b), ("stage 1", L, lc)
        exp_plane, exp_bands = port.closed_loop(pl, L, lc, t, 84, 0, 84)
        W = ric.Wavelet2D(w, h, L, lc)
        W.SetWeight(t)
        W.Transform(pl, w, t)
        buf = np.zeros(w * h * 8 + 4096, np.uint8)
        m = ric.MuxCodec(buf, first_word=0)
        W.CodeBand(m, 84, 0)
        m.endCoding()
        W.TSUQi(84)
        for a, b in zip(W.bands(), exp_bands):
            assert np.array_equal(a, b), ("closed loop bands", L, lc)
        out = np.zeros((h, w), np.int16)
        W.TransformI(out, w, t)
        assert np.array_equal(out, exp_plane), ("closed loop plane", L, lc)


@pytest.mark.parametrize("e", G["small"], ids=[e["name"] for e in G["small"]])
def test_small_golden_split_encoder(ric, e):
    """ric_codec_set_host_threads: bands modelled in parallel, the stream
    written in coding order from their event lists -- the golden bytes"""
    pix = ric.synth(e["w"], e["h"], e["channels"], e["frame"])
    c = ric.Codec(e["w"], e["h"], e["channels"])
    c.set_host_threads(4)
    assert c.compress(pix, e["q"], e["trans"]) == open(os.path.join(GOLD, e["name"] + ".ric"), "rb").read()


@pytest.mark.parametrize("name", ["C3_7680x4320_q9", "C3rgb_7680x4320_q9", "lossless53_1001x603"])
def test_full_size_split_encoder(ric, name):
    e = large(name)
    pix = ric.synth(e["w"], e["h"], e["channels"], e["frame"])
    c = ric.Codec(e["w"], e["h"], e["channels"])
    c.set_host_threads(8)
    for _ in range(2):                         # event buffers reused across frames
        r = c.compress(pix, e["q"], e["trans"])
        assert len(r) == e["ric_bytes"] and sha(r) == e["ric_sha256"]


def test_codeband_split_encoder(ric, port):
    """CWavelet2D::CodeBand over the split (ric_wavelet_set_host_threads),
    with the band state the API leaves (closed loop)"""
    w, h, t, L, lc = 300, 220, 0, 5, 1
    pl = O.gray_plane(ric.synth(w, h, 1, 6)[0], 9)
    exp_plane, exp_bands = port.closed_loop(pl, L, lc, t, 96, 36, 96)
    W = ric.Wavelet2D(w, h, L, lc)
    W.SetWeight(t)
    W.set_host_threads(3)
    W.Transform(pl, w, t)
    buf = np.zeros(w * h * 4 + 4096, np.uint8)
    m = ric.MuxCodec(buf, first_word=0)
    W.CodeBand(m, 96, 36)
    m.endCoding()
    W.TSUQi(96)
    for a, b in zip(W.bands(), exp_bands):
        assert np.array_equal(a, b)
    out = np.zeros((h, w), np.int16)
    W.TransformI(out, w, t)
    assert np.array_equal(out, exp_plane)
    # the stream: the one-thread CodeBand's bytes
    W1 = ric.Wavelet2D(w, h, L, lc)
    W1.SetWeight(t)
    W1.Transform(pl, w, t)
    buf1 = np.zeros_like(buf)
    m1 = ric.MuxCodec(buf1, first_word=0)
    W1.CodeBand(m1, 96, 36)
    m1.endCoding()
    assert np.array_equal(buf, buf1)


def test_band_operations(ric):
    """CBand's TSUQ / TSUQi / Mean / Add / Clear on single bands, on the
    device (ric_band_*), against numpy restatements of src/lib/band.h:65-141"""
    w, h = 257, 130
    pl = O.gray_plane(ric.synth(w, h, 1, 3)[0], 9)
    W = ric.Wavelet2D(w, h, 5, 1)
    W.SetWeight(0)
    W.Transform(pl, w, 0)
    raw = W.bands()
    f32 = np.float32
    for i in range(W.band_count()):
        _, _, isint, wt = W.band_info(i)
        # TSUQ(96, 0.6)
        Q = int(f32(96) / f32(wt)) or 1
        iQ = 65536 // Q
        T = int(f32(0.6) * f32(Q))
        T = T if isint else int(np.int16(T))
        v = raw[i].astype(np.int64)
        dead = ((v + T) & 0xFFFFFFFF) <= ((2 * T) & 0xFFFFFFFF)
        q = (((v * iQ + 32768) & 0xFFFFFFFF).astype(np.uint32).view(np.int32) >> 16).astype(np.int64)
        q = q if isint else q.astype(np.int16).astype(np.int64)
        exp = np.where(dead, 0, q)
        cnt, mx, mn = W.band_tsuq(i, 96, 0.6)
        got = W.bands()[i]
        assert np.array_equal(got, exp), i
        assert cnt == int((~dead).sum()) and mx == max(0, int(exp.max())) and mn == min(0, int(exp.min())), i
        # Mean's sums
        s, ss = W.band_sums(i)
        e = exp.astype(np.int64)
        assert s == int(e.sum())
        assert ss == int(((e * e) & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64).sum())
        # TSUQi(40)
        W.band_tsuqi(i, 40)
        qi = 40 if isint else int(np.int16(40))
        qi = int(f32(qi) / f32(wt))
        qi = (qi if isint else int(np.int16(qi))) or 1
        e2 = e * qi
        e2 = e2.astype(np.int32) if isint else e2.astype(np.int16)
        assert np.array_equal(W.bands()[i], e2.astype(np.int64)), i
        # Add(-3), Clear
        W.band_add(i, -3)
        e3 = e2.astype(np.int64) - 3
        e3 = e3.astype(np.int32) if isint else e3.astype(np.int16)
        assert np.array_equal(W.bands()[i], e3.astype(np.int64)), i
    W.band_clear(0)
    assert not W.bands()[0].any()
