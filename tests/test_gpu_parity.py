"""GPU parity: the HIP path through the C-ABI against the CPU oracle
(oracle/ric_oracle.c, itself pinned to the reference library and the golden
vectors).  Integer work: every comparison is bit-exact."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIZES = [(512, 512), (33, 47), (1001, 603), (17, 16), (240, 135), (64, 64), (129, 77), (1000, 600)]


def _plane(w, h, q=9, frame=0):
    return O.gray_plane(O.synth(w, h, 1, frame)[0], q)


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("trans", [0, 1])
def test_forward_bands(ric, port, w, h, trans):
    pl = _plane(w, h)
    W = ric.Wavelet2D(w, h, 5, 1)
    W.SetWeight(trans)
    W.Transform(pl, w, trans)
    got = W.bands()
    exp = port.bands(pl, 5, 1, trans, 0)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert np.array_equal(g, e), "band %d differs (%d mismatches)" % (i, int((g != e).sum()))


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("trans", [0, 1])
def test_inverse(ric, port, w, h, trans):
    # inverse of the oracle's forward bands (exact reconstruction path)
    pl = _plane(w, h)
    bands = port.bands(pl, 5, 1, trans, 0)
    W = ric.Wavelet2D(w, h, 5, 1)
    for i, b in enumerate(bands):
        W.write_band(i, b)
    out = np.zeros((h, w), np.int16)
    W.TransformI(out, w, trans)
    exp = np.zeros((h, w), np.int16)
    flat = np.concatenate([b.ravel() for b in bands]).astype(np.int32)
    port.lib.ricor_inverse(flat.ctypes.data, w, h, 5, 1, trans, exp.ctypes.data)
    assert np.array_equal(out, exp), int((out != exp).sum())


@pytest.mark.parametrize("w,h,q,t", [(512, 512, 9, 0), (512, 512, 0, 1), (33, 47, 9, 0), (1001, 603, 0, 1),
                                     (1000, 600, 5, 0), (64, 64, 31, 0), (129, 77, 1, 1), (640, 480, 20, 0)])
def test_ric_gray(ric, port, w, h, q, t):
    pix = O.synth(w, h, 1)
    C = ric.Codec(w, h, 1)
    got = C.compress(pix, q, t)
    exp = port.encode_ric(pix, q, t)
    assert got == exp
    pg, plg = C.decompress(exp)
    pe, ple = port.decode_ric(exp)
    assert np.array_equal(plg, ple)
    assert np.array_equal(pg, pe)


@pytest.mark.parametrize("w,h,q,t", [(512, 512, 9, 0), (96, 80, 0, 1), (300, 201, 12, 0)])
def test_ric_rgb(ric, port, w, h, q, t):
    pix = O.synth(w, h, 3)
    C = ric.Codec(w, h, 3)
    got = C.compress(pix, q, t)
    exp = port.encode_ric(pix, q, t)
    assert got == exp
    pg, plg = C.decompress(exp)
    pe, ple = port.decode_ric(exp)
    assert np.array_equal(plg, ple)
