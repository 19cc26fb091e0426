"""The clean-room oracle against the reference library compiled in place
(oracle/_ref).  Skipped where the reference build is absent."""
import numpy as np
import pytest

from oracle import oracle as O

REF = O.ref()
pytestmark = pytest.mark.skipif(REF is None, reason="oracle/_ref not built (reference sources absent)")

SIZES = [(8, 8), (16, 16), (17, 23), (33, 47), (64, 48), (100, 101), (129, 77), (255, 130), (1001, 603)]


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("t", [0, 1])
@pytest.mark.parametrize("stage", [0, 1, 2])
def test_bands(w, h, t, stage):
    pl = O.gray_plane(O.synth(w, h, 1, 3)[0], 9)
    # the top level is always `short` in the reference callers (Transform<short> only);
    # level_chg >= levels would make it int, which the reference mis-handles
    for L, lc in [(5, 1), (3, -1), (4, 2)]:
        a = O.port().bands(pl, L, lc, t, stage, 96, 36)
        b = REF.bands(pl, L, lc, t, stage, 96, 36)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("w,h", [(64, 48), (129, 77), (300, 220)])
@pytest.mark.parametrize("t", [0, 1])
@pytest.mark.parametrize("L,lc", [(5, 1), (3, 0)])
def test_closed_loop(w, h, t, L, lc):
    """CodeBand -> TSUQi -> TransformI on the bands CodeBand leaves behind
    (the video driver's loop, src/lib/rududucodec.cpp:67-74)."""
    pl = O.gray_plane(O.synth(w, h, 1, 6)[0], 9)
    a, ab = O.port().closed_loop(pl, L, lc, t, 96, 36, 96)
    b, bb = REF.closed_loop(pl, L, lc, t, 96, 36, 96)
    assert np.array_equal(a, b)
    for x, y in zip(ab, bb):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("q", [0, 1, 5, 9, 20, 31])
@pytest.mark.parametrize("t", [0, 1])
@pytest.mark.parametrize("w,h", [(64, 48), (129, 77), (200, 113)])
def test_ric_gray(q, t, w, h):
    pix = O.synth(w, h, 1, q)
    a = O.port().encode_ric(pix, q, t)
    assert a == REF.encode_ric(pix, q, t)
    assert np.array_equal(O.port().decode_ric(a)[1], REF.decode_ric(a)[1])


@pytest.mark.parametrize("q,t", [(0, 1), (9, 0), (31, 0), (3, 1)])
def test_ric_rgb(q, t):
    pix = O.synth(96, 72, 3, q)
    a = O.port().encode_ric(pix, q, t)
    assert a == REF.encode_ric(pix, q, t)
    assert np.array_equal(O.port().decode_ric(a)[1], REF.decode_ric(a)[1])


def test_dither_decode():
    pix = O.synth(80, 60, 1, 2)
    a = REF.encode_ric(pix, 12, 0)
    assert np.array_equal(O.port().decode_ric(a, dither=True)[0], REF.decode_ric(a, dither=True)[0])


def test_haar_even_sizes():
    pix = O.synth(128, 96, 1, 5)     # every level even: the reference is deterministic
    a = O.port().encode_ric(pix, 9, 2)
    assert a == REF.encode_ric(pix, 9, 2)
    assert np.array_equal(O.port().decode_ric(a)[1], REF.decode_ric(a)[1])


@pytest.mark.parametrize("w,h", [(64, 48), (300, 220), (1001, 603)])
@pytest.mark.parametrize("t", [0, 1])
def test_stats_restatement(w, h, t):
    """oracle.band_variance / set_weight (the numbers CWavelet2D::Stats
    prints) against the reference's CBand::Mean on its own bands."""
    import ctypes
    pl = O.gray_plane(O.synth(w, h, 1, 5)[0], 9)
    f = REF.lib.ricref_stats
    f.restype = ctypes.c_long
    f.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p]
    out = np.zeros(64, np.float32)
    n = f(pl.ctypes.data, w, h, 5, 1, t, out.ctypes.data)
    bands = REF.bands(pl, 5, 1, t, 0)
    assert n == len(bands)
    wts = O.set_weight(n, t)
    for i, b in enumerate(bands):
        assert O.band_variance(b, wts[i]) == out[i], i


@pytest.mark.parametrize("kind", ["uniform", "alt", "ramp"])
@pytest.mark.parametrize("w,h", [(64, 48), (129, 77), (96, 64)])
@pytest.mark.parametrize("t", [0, 1])
def test_full_range_planes(kind, w, h, t):
    """forward band dumps (stages 0-2) and the closed loop on planes whose
    lifting sums leave the 16-bit range"""
    pl = O.full_range_plane(w, h, w * h, kind)
    for L, lc in [(3, 0), (5, 1)]:
        for stage in (0, 1, 2):
            for x, y in zip(O.port().bands(pl, L, lc, t, stage, 96, 36), REF.bands(pl, L, lc, t, stage, 96, 36)):
                assert np.array_equal(x, y), (L, lc, stage)
        a, ab = O.port().closed_loop(pl, L, lc, t, 84, 0, 84)
        b, bb = REF.closed_loop(pl, L, lc, t, 84, 0, 84)
        assert np.array_equal(a, b), (L, lc)
