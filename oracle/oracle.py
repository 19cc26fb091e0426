"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for the two CPU checkers:
  * ``port``: liboracle.so, the clean-room C restatement (oracle/ric_oracle.c);
  * ``ref``:  _ref/libricref.so, the unmodified reference library compiled
    from /root/reference/src/lib by oracle/Makefile (absent when the reference
    sources were not available at build time).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  Both libraries expose the same entry points (ricor_* / ricref_*),
so a ``Checker`` wraps either one.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PORT_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libricref.so")

_P = ctypes.c_void_p
_L = ctypes.c_long
_I = ctypes.c_int


def _ptr(a):
    return a.ctypes.data_as(_P) if a is not None else None


class Checker:
    """One CPU implementation of the .ric path (port or reference)."""

    def __init__(self, path, prefix):
        self.path = path
        self.lib = ctypes.CDLL(path)
        self.prefix = prefix
        sig = {
            "layout": (_I, [_I, _I, _I, _I, _P]),
            "bands": (_L, [_P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
            "encode_planes": (_L, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _L]),
            "decode_planes": (_L, [_P, _L, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
            "encode_ric": (_L, [_P, _I, _I, _I, _I, _I, _P, _L]),
            "decode_ric": (_L, [_P, _L, _I, _P, _P, _P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(self.lib, prefix + name)
            f.restype, f.argtypes = res, args

    def _f(self, name):
        return getattr(self.lib, self.prefix + name)

    def layout(self, w, h, levels=5, lc=1):
        n = self._f("layout")(w, h, levels, lc, None)
        out = np.zeros(3 * n, np.int32)
        self._f("layout")(w, h, levels, lc, _ptr(out))
        return out.reshape(n, 3)

    def bands(self, plane, levels=5, lc=1, trans=0, stage=0, quant=0, lam=0):
        plane = np.ascontiguousarray(plane, np.int16)
        h, w = plane.shape
        lay = self.layout(w, h, levels, lc)
        total = int((lay[:, 0] * lay[:, 1]).sum())
        out = np.zeros(total, np.int32)
        n = self._f("bands")(_ptr(plane), w, h, levels, lc, trans, stage, quant, lam, _ptr(out))
        assert n == total
        return split_bands(out, lay)

    def encode_planes(self, planes, levels, lc, trans, quants, lambdas):
        planes = np.ascontiguousarray(planes, np.int16)
        c, h, w = planes.shape
        cap = w * h * c * 4 + 4096
        out = np.zeros(cap, np.uint8)
        q = np.asarray(quants, np.int32)
        lm = np.asarray(lambdas, np.int32)
        n = self._f("encode_planes")(_ptr(planes), c, w, h, levels, lc, trans, _ptr(q), _ptr(lm), _ptr(out), cap)
        assert n > 0
        return out[:n].tobytes()

    def decode_planes(self, buf, nplanes, w, h, levels, lc, trans, quants, want_bands=False):
        b = np.frombuffer(buf, np.uint8).copy()
        out = np.zeros((nplanes, h, w), np.int16)
        q = np.asarray(quants, np.int32)
        bands = None
        if want_bands:
            lay = self.layout(w, h, levels, lc)
            bands = np.zeros(int((lay[:, 0] * lay[:, 1]).sum()), np.int32)
        self._f("decode_planes")(_ptr(b), len(buf), nplanes, w, h, levels, lc, trans, _ptr(q), _ptr(out), _ptr(bands))
        if want_bands:
            return out, split_bands(bands, self.layout(w, h, levels, lc))
        return out

    def encode_ric(self, pix, q, trans):
        pix = np.ascontiguousarray(pix, np.uint8)
        c, h, w = pix.shape
        cap = w * h * c * 4 + 4096
        out = np.zeros(cap, np.uint8)
        n = self._f("encode_ric")(_ptr(pix), w, h, c, q, trans, _ptr(out), cap)
        assert n > 0
        return out[:n].tobytes()

    def closed_loop(self, plane, levels, lc, trans, quant, lam, dq):
        """Transform -> CodeBand -> TSUQi(dq) -> TransformI on one int16 plane
        (src/lib/rududucodec.cpp:67-74): (reconstructed plane, bands after TSUQi)."""
        plane = np.ascontiguousarray(plane, np.int16)
        h, w = plane.shape
        lay = self.layout(w, h, levels, lc)
        bands = np.zeros(int((lay[:, 0] * lay[:, 1]).sum()), np.int32)
        out = np.zeros((h, w), np.int16)
        f = self._f("closed_loop")
        f.restype = _L
        f.argtypes = [_P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P]
        f(_ptr(plane), w, h, levels, lc, trans, quant, lam, dq, _ptr(out), _ptr(bands))
        return out, split_bands(bands, lay)

    def decode_ric(self, ric, dither=False):
        b = np.frombuffer(ric, np.uint8).copy()
        dims = np.zeros(5, np.int32)
        rc = self._f("decode_ric")(_ptr(b), len(ric), int(dither), None, None, _ptr(dims))
        if rc < 0:
            raise ValueError("bad magic (reference throws BAD_MAGIC=%d)" % -rc)
        w, h, c = int(dims[0]), int(dims[1]), int(dims[2])
        pix = np.zeros((c, h, w), np.uint8)
        planes = np.zeros((c, h, w), np.int16)
        self._f("decode_ric")(_ptr(b), len(ric), int(dither), _ptr(planes), _ptr(pix), None)
        return pix, planes


def split_bands(flat, lay):
    out, off = [], 0
    for dx, dy, _ in lay:
        n = int(dx) * int(dy)
        out.append(flat[off:off + n].reshape(int(dy), int(dx)))
        off += n
    return out


_port = None
_ref = None


def port():
    """The clean-room C restatement (always available once built)."""
    global _port
    if _port is None:
        _port = Checker(PORT_SO, "ricor_")
        lib = _port.lib
        lib.ricor_synth.restype = None
        lib.ricor_synth.argtypes = [_I, _I, _I, _I, _P]
        lib.ricor_quants.restype = ctypes.c_short
        lib.ricor_quants.argtypes = [_I]
        lib.ricor_inverse.restype = _L
        lib.ricor_inverse.argtypes = [_P, _I, _I, _I, _I, _I, _P]
    return _port


def ref():
    """The reference library itself, or None when it was not built."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        _ref = Checker(REF_SO, "ricref_")
    return _ref


def synth(w, h, channels=1, frame=0):
    """SURVEY.md §8(d) synthetic image, (channels, h, w) uint8."""
    out = np.zeros((channels, h, w), np.uint8)
    port().lib.ricor_synth(w, h, channels, frame, _ptr(out))
    return out


def quants(idx):
    return int(port().lib.ricor_quants(idx))


def set_weight(n_bands, trans, base=1.0):
    """CWavelet2D::SetWeight (src/lib/wavelet2d.cpp:1009-1032) in float32:
    the weights of the canonical band order (per level D, H, V; then L)."""
    f = np.float32
    scale = f(1.149604398) * f(1.149604398) if trans == 0 else f(2.0)
    out, nlev = [], (n_bands - 1) // 3
    D, V, H, L = f(base) / scale, f(base), f(base), f(base) * scale
    for l in range(nlev):
        if l > 0:
            D, V = V, L
            H, L = V, V * scale
        out += [D, H, V]
    return out + [L]


def band_variance(band, weight):
    """CBand::Mean's variance (src/lib/band.h:116-132) with the reference's
    C arithmetic: int products, int64 sums (wrapping), the sample count
    squared in unsigned, float32 arithmetic."""
    v = band.astype(np.int64)
    s = int(v.sum())
    ss = int(((v * v) & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64).sum())
    d = ((ss - s * s) + (1 << 63)) % (1 << 64) - (1 << 63)
    n = (band.shape[0] * band.shape[1]) & 0xFFFFFFFF
    w = np.float32(weight)
    return np.float32(np.float32(d) * w * w / np.float32((n * n) & 0xFFFFFFFF))


def gray_plane(pix, q):
    """Level shift of src/ric/ric.cpp:144-148 for one gray plane."""
    p = pix.astype(np.int32) - 128
    return (p << 4 if q else p).astype(np.int16)


def full_range_plane(w, h, seed, kind):
    """int16 planes that push the 9/7 lifting past 16 bits: the mult08 of a
    sum runs in int in the reference (the template deduces C = int,
    src/lib/wavelet2d.cpp:336), so a restatement that wraps the sum differs"""
    rng = np.random.default_rng(seed)
    if kind == "uniform":
        return rng.integers(-32768, 32768, (h, w)).astype(np.int16)
    if kind == "alt":                                   # extreme alternating pattern
        y, x = np.mgrid[0:h, 0:w]
        return np.where(((x + y) % 2) == 0, 32767, -32768).astype(np.int16)
    y, x = np.mgrid[0:h, 0:w]                           # large smooth ramp + noise
    return np.clip(30000 * np.sin(x / 7.0) * np.cos(y / 5.0) + rng.normal(0, 3000, (h, w)), -32768, 32767).astype(np.int16)
