"""The video codec's checker and its host serial half, on the CPU.

* oracle/_ref/ricvid_ref (the reference video codec's classes compiled from
  /root/reference/src/lib, oracle/ref_video.cpp) reproduces the committed
  golden hashes (tests/golden/video.json) -- this pins the checker build;
* the product's motion-vector decoder (entropy.cpp mv_decode: COBMC::decode,
  src/lib/obmc.cpp:393-440, with the adaptive CHuffCodec) reads the
  reference's own streams back to the reference's vectors;
* mv_encode -> mv_decode round trips fields that reach every code path
  (intra blocks, zero residuals, the huff_x / huff_y escapes, the linear
  Golomb tail, Huffman rebuilds)."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import video_seq
import hostcoder

HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "video.json")))


def _sha(x):
    return hashlib.sha256(bytes(x)).hexdigest()


def _ref_available():
    if not os.path.exists(video_seq.REF_BIN):
        pytest.skip("oracle/_ref/ricvid_ref not built (make -C oracle with the reference sources)")


@pytest.mark.parametrize("cfg", G["sequences"], ids=lambda c: "%dx%d_q%d" % (c["w"], c["h"], c["q"]))
def test_ref_video_matches_golden(cfg, tmp_path):
    _ref_available()
    seq = video_seq.sequence(cfg["w"], cfg["h"], cfg["frames"], cfg["seed"])
    fr = video_seq.ref_run(seq, cfg["q"], tmp_path)
    assert [_sha(f["stream"]) for f in fr] == cfg["stream_sha256"]
    assert [_sha(f["enc"].tobytes()) for f in fr] == cfg["enc_sha256"]
    assert [_sha(f["dec"].tobytes()) for f in fr] == cfg["dec_sha256"]
    assert [_sha(f["mv"].tobytes()) for f in fr] == cfg["mv_sha256"]


def _mv_lib():
    L = hostcoder.lib()
    L.hc_mv_decode.restype = ctypes.c_long
    L.hc_mv_decode.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.hc_mv_encode.restype = ctypes.c_long
    L.hc_mv_encode.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long]
    return L


def _decode(stream, dimx, dimy):
    b = np.zeros(len(stream) + 64, np.uint8)
    b[:len(stream)] = np.frombuffer(stream, np.uint8)
    mv = np.zeros((dimy, dimx), np.uint32)
    _mv_lib().hc_mv_decode(b.ctypes.data, b.size, dimx, dimy, mv.ctypes.data)
    return mv


@pytest.mark.parametrize("cfg", G["sequences"][:2], ids=lambda c: "%dx%d" % (c["w"], c["h"]))
def test_mv_decoder_reads_reference_streams(cfg, tmp_path):
    _ref_available()
    seq = video_seq.sequence(cfg["w"], cfg["h"], cfg["frames"], cfg["seed"])
    fr = video_seq.ref_run(seq, cfg["q"], tmp_path)
    n_inter = 0
    for k, f in enumerate(fr):
        if not f["stream"][0] & 0x80:            # key frame: no vectors in the stream
            continue
        got = _decode(f["stream"], cfg["w"] >> 3, cfg["h"] >> 3)
        assert np.array_equal(got, f["mv"]), "frame %d" % k
        n_inter += 1
    assert n_inter >= 3


def _field(dimx, dimy, seed):
    rng = np.random.default_rng(seed)
    x = rng.integers(-40, 40, (dimy, dimx))
    y = rng.integers(-40, 40, (dimy, dimx))
    big = rng.random((dimy, dimx)) < 0.05                    # past the huff_x/y escape and the Golomb tail
    x[big] = rng.integers(-3000, 3000, int(big.sum()))
    same = rng.random((dimy, dimx)) < 0.3
    x[same], y[same] = 0, 0
    mv = (x.astype(np.uint32) & 0xFFFF) | ((y.astype(np.uint32) & 0xFFFF) << 16)
    mv[rng.random((dimy, dimx)) < 0.05] = 0x80008000          # MV_INTRA
    return mv.astype(np.uint32)


@pytest.mark.parametrize("dimx,dimy,seed", [(16, 12, 1), (160, 90, 2), (2, 2, 3), (40, 3, 4)])
def test_mv_coder_roundtrip(dimx, dimy, seed):
    mv = _field(dimx, dimy, seed)
    cap = mv.size * 16 + 4096
    out = np.zeros(cap, np.uint8)
    n = _mv_lib().hc_mv_encode(mv.ctypes.data, dimx, dimy, out.ctypes.data, cap)
    assert n > 0
    assert np.array_equal(_decode(out[:n].tobytes(), dimx, dimy), mv)
