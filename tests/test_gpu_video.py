"""The reference video codec's coding loop (src/lib/rududucodec.cpp) on the GPU
against the reference library itself (oracle/_ref, compiled from
/root/reference/src/lib by oracle/Makefile).

test_video_intra_*: tests/native/video_intra.cpp, ONE source built on the GPU
drop-in (include/rududu_gpu.hpp) and against the reference's headers: the
CMuxCodec(0, 0) + initCoder / initDecoder per frame, CWavelet2D(w, h, 3),
Transform -> CodeBand -> TSUQi -> TransformI on CImage-style bordered planes
with the video quants() table.  Streams and planes must be byte-identical."""
import os
import subprocess

import json

import numpy as np
import pytest

import video_seq

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SHIM_BIN = os.path.join(HERE, "native", "video_intra")
REF_BIN = os.path.join(REPO, "oracle", "_ref", "video_intra_ref")


def _planes(w, h, n, seed):
    """n frames of 3 int16 planes in the video codec's scale (Y << 4, Co/Cg << 3:
    src/lib/image.cpp:113-117) from the synthetic generator, shifted per frame."""
    import ric_amd
    out = []
    for f in range(n):
        rgb = ric_amd.synth(w + 16, h + 16, 3, seed + f // 4)[:, (3 * f) % 16:(3 * f) % 16 + h, (5 * f) % 16:(5 * f) % 16 + w]
        r, g, b = (rgb[i].astype(np.int32) for i in range(3))
        co = r - b
        y = b + (co >> 1)
        cg = g - y
        y = y + (cg >> 1) - 128
        out += [(y << 4).astype(np.int16), (co << 3).astype(np.int16), (cg << 3).astype(np.int16)]
    return np.stack(out)


def _byte_diff(a, b):
    """where two byte strings first differ (pytest's own diff of MB-sized
    bytes takes minutes)"""
    n = min(len(a), len(b))
    d = np.nonzero(np.frombuffer(a[:n], np.uint8) != np.frombuffer(b[:n], np.uint8))[0]
    return "lengths %d vs %d, first difference at %s" % (len(a), len(b), int(d[0]) if d.size else n)


def _run(binary, w, h, q, n, planes, tmp):
    src = os.path.join(tmp, "in.i16")
    dst = os.path.join(tmp, os.path.basename(binary) + ".bin")
    planes.astype(np.int16).tofile(src)
    subprocess.run([binary, str(w), str(h), str(q), str(n), src, dst], check=True, timeout=120)
    return open(dst, "rb").read()


def _frames(blob, w, h, n):
    """split video_intra's output into per-frame (stream, enc planes, dec planes, dec size)"""
    out, o = [], 0
    npl = 3 * w * h * 2
    for _ in range(n):
        size = int(np.frombuffer(blob, np.uint32, 1, o)[0])
        o += 4
        s = blob[o:o + size + 2]
        o += size + 2
        e = np.frombuffer(blob, np.int16, 3 * w * h, o).reshape(3, h, w)
        o += npl
        d = np.frombuffer(blob, np.int16, 3 * w * h, o).reshape(3, h, w)
        o += npl
        ds = int(np.frombuffer(blob, np.uint32, 1, o)[0])
        o += 4
        out.append((s, e, d, ds))
    assert o == len(blob)
    return out


# q is CRududuCodec::quant: quants(q + 20) is the quantiser and quants(q + 12)
# the RD lambda, so q >= -12 (below, quants reads its table at a negative
# index: undefined in the reference); q = -12 gives the densest streams
# (quants(8) = 84), testmotion.cpp uses 20 (quants(40) = 7132)
@pytest.mark.parametrize("w,h,q,n", [(128, 96, -10, 3), (160, 120, -12, 2), (200, 72, 0, 2), (97, 61, -5, 2),
                                     (352, 288, -11, 3), (64, 48, 20, 2)])
def test_video_intra_matches_reference(ric, tmp_path, w, h, q, n):
    if not os.path.exists(REF_BIN):
        pytest.fail("oracle/_ref/video_intra_ref not built (make -C oracle with /root/reference present)")
    planes = _planes(w, h, n, 300 + w)
    got = _run(SHIM_BIN, w, h, q, n, planes, str(tmp_path))
    want = _run(REF_BIN, w, h, q, n, planes, str(tmp_path))
    gf, wf = _frames(got, w, h, n), _frames(want, w, h, n)
    for k, (g, e) in enumerate(zip(gf, wf)):
        assert g[0] == e[0], "frame %d stream: %s" % (k, _byte_diff(g[0], e[0]))
        assert np.array_equal(g[1], e[1]), "frame %d encoder reconstruction" % k
        assert np.array_equal(g[2], e[2]), "frame %d decoder planes" % k
        assert g[3] == e[3], "frame %d decoder getSize" % k
    assert got == want, _byte_diff(got, want)


GV = json.load(open(os.path.join(HERE, "golden", "video.json")))


def _first_diff(a, b):
    d = np.argwhere(a != b)
    return None if d.size == 0 else (tuple(int(x) for x in d[0]), int(a[tuple(d[0])]), int(b[tuple(d[0])]), len(d))


def _check_sequence(ric, w, h, q, n, seed, tmp_path, host_threads=1):
    """CRududuCodec on the GPU vs the reference's classes (oracle/_ref/ricvid_ref),
    frame by frame: stream bytes, encoder output image (with its border: the
    next frame's quarter-pel pass reads it), motion field, decoder output."""
    if not os.path.exists(video_seq.REF_BIN):
        pytest.fail("oracle/_ref/ricvid_ref not built (make -C oracle with /root/reference present)")
    seq = video_seq.sequence(w, h, n, seed)
    want = video_seq.ref_run(seq, q, tmp_path)
    enc = ric.VideoCodec(True, w, h)
    dec = ric.VideoCodec(False, w, h)
    enc.quant = q
    dec.quant = q
    if host_threads > 1:
        enc.set_host_threads(host_threads)
    B = video_seq.BORDER
    for k in range(n):
        e = want[k]
        s = enc.encode(seq[k])
        assert np.array_equal(enc.motion(), e["mv"]), "frame %d motion field: %s" % (k, _first_diff(enc.motion(), e["mv"]))
        bo = enc.output(border=True)
        assert np.array_equal(bo[:, B:B + h, B:B + w], e["enc"]), \
            "frame %d encoder image: %s" % (k, _first_diff(bo[:, B:B + h, B:B + w], e["enc"]))
        assert np.array_equal(bo, e["bordered"]), "frame %d encoder image border: %s" % (k, _first_diff(bo, e["bordered"]))
        assert s == e["stream"], "frame %d stream: %s" % (k, _byte_diff(s, e["stream"]))
        assert dec.decode(s) == e["dsize"], "frame %d decoder getSize" % k
        assert np.array_equal(dec.output(), e["dec"]), "frame %d decoder image: %s" % (k, _first_diff(dec.output(), e["dec"]))


@pytest.mark.parametrize("cfg", GV["sequences"], ids=lambda c: "%dx%d_q%d" % (c["w"], c["h"], c["q"]))
def test_video_golden_sequences(ric, cfg, tmp_path):
    _check_sequence(ric, cfg["w"], cfg["h"], cfg["q"], cfg["frames"], cfg["seed"], tmp_path)


@pytest.mark.parametrize("w,h,q,n,seed", [(68, 44, 4, 3, 11), (333, 141, -12, 3, 12), (1280, 720, 20, 3, 13)])
def test_video_sequences(ric, w, h, q, n, seed, tmp_path):
    """odd and non-multiple-of-8 sizes (the OBMC grid does not cover the
    frame), the finest quantiser, and testmotion.cpp's 1280x720 at quant 20"""
    _check_sequence(ric, w, h, q, n, seed, tmp_path)


def test_video_sequence_split_encoder(ric, tmp_path):
    """the encoder's serial stage with its bands modelled in parallel
    (ric_video_set_host_threads): the same streams, 12 frames across a key"""
    _check_sequence(ric, 320, 240, 6, 12, 31, tmp_path, host_threads=6)


COMPAT_BIN = os.path.join(HERE, "native", "video_compat")


@pytest.mark.parametrize("w,h,q,n,seed", [(128, 96, -5, 12, 5), (176, 144, 20, 4, 21)])
def test_video_compat_caller(ric, w, h, q, n, seed, tmp_path):
    """tests/native/video_compat.cpp -- testmotion.cpp's calls (CRududuCodec
    encode / decode, quant, CImage::psnr, outputYV12<char, false>) over the
    GPU drop-in: the same streams, sizes and YV12 output as the reference."""
    seq = video_seq.sequence(w, h, n, seed)
    want = video_seq.ref_run(seq, q, tmp_path)
    src = os.path.join(str(tmp_path), "compat.rgb")
    dst = os.path.join(str(tmp_path), "compat.bin")
    np.ascontiguousarray(seq).tofile(src)
    subprocess.run([COMPAT_BIN, str(w), str(h), str(q), str(n), src, dst], check=True, timeout=300)
    blob, o = open(dst, "rb").read(), 0
    for k in range(n):
        size = int(np.frombuffer(blob, np.uint32, 1, o)[0]); o += 4
        stream = blob[o:o + size + 2]; o += size + 2
        dsize = int(np.frombuffer(blob, np.uint32, 1, o)[0]); o += 4
        yv = blob[o:o + w * h * 3 // 2]; o += w * h * 3 // 2
        psnr = np.frombuffer(blob, np.float32, 6, o).reshape(2, 3); o += 24
        e = want[k]
        assert size == e["size"] and stream == e["stream"], "frame %d stream: %s" % (k, _byte_diff(stream, e["stream"]))
        assert dsize == e["dsize"], "frame %d decode() return" % k
        assert yv == e["yv12"], "frame %d outputYV12: %s" % (k, _byte_diff(yv, e["yv12"]))
        # CImage::psnr (src/lib/image.cpp:248-265) of the origin against both outputs
        r, g_, b = (seq[k][i].astype(np.int32) for i in range(3))
        co = r - b
        y = b + (co >> 1)
        cg = g_ - y
        y = y + (cg >> 1) - 128
        origin = np.stack([y * 16, co * 8, cg * 8])[:, ::-1, :]       # inputSGI: bottom row first
        for side, planes in ((0, e["enc"]), (1, e["dec"])):
            mse = ((planes.astype(np.int64) - origin) ** 2).reshape(3, -1).sum(1) / (w * h)
            ref_psnr = (10.0 * (np.log(float(1 << 24)) - np.log(mse)) / np.log(10.0)).astype(np.float32)
            np.testing.assert_allclose(psnr[side], ref_psnr, rtol=1e-6)
    assert o == len(blob)
