"""ctypes binding of tests/native/libhostcoder.so: the product's host serial
coder (rududu-image-codec_amd/csrc/{entropy,encoder,decoder}.cpp) driven on the
CPU from band dumps, so the serial stage is testable without a GPU."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "native", "libhostcoder.so")
_V, _I, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO) or os.path.getmtime(SO) < max(
                os.path.getmtime(os.path.join(HERE, "native", f)) for f in os.listdir(os.path.join(HERE, "native"))
                if f.endswith(".cpp")):
            os.system("make -s -C %s" % os.path.join(HERE, "native"))
        L = ctypes.CDLL(SO)
        L.hc_encode.restype = _L
        L.hc_encode.argtypes = [_V, _L, _I, _I, _I, _I, _I, _V, _L, _V]
        L.hc_encode_rec.restype = _L
        L.hc_encode_rec.argtypes = [_V, _L, _I, _I, _I, _I, _I, _V, _L, _V, _V]
        L.hc_encode_rec_split.restype = _L
        L.hc_encode_rec_split.argtypes = [_V, _L, _I, _I, _I, _I, _I, _V, _L, _I, _V, _V, _V]
        L.hc_encode_rec_compact.restype = _L
        L.hc_encode_rec_compact.argtypes = [_V, _L, _I, _I, _I, _I, _I, _V, _L]
        L.hc_decode_compact.restype = _L
        L.hc_decode_compact.argtypes = [_V, _L, _I, _I, _I, _I, _I, _V, _V]
        L.hc_decode.restype = _L
        L.hc_decode.argtypes = [_V, _L, _I, _I, _I, _I, _I, _V, _V]
        _lib = L
    return _lib


def encode(bands_flat, w, h, levels, lc, records=True):
    """bands_flat: stage-1 canonical dump (int32) of ONE plane -> coder buffer bytes."""
    b = np.ascontiguousarray(bands_flat, np.int32)
    cap = w * h * 4 + 4096
    out = np.zeros(cap, np.uint8)
    s1, s2 = ctypes.c_double(), ctypes.c_double()
    if records:
        n = lib().hc_encode_rec(b.ctypes.data, b.size, 1, w, h, levels, lc, out.ctypes.data, cap,
                                ctypes.byref(s1), ctypes.byref(s2))
    else:
        n = lib().hc_encode(b.ctypes.data, b.size, 1, w, h, levels, lc, out.ctypes.data, cap, ctypes.byref(s1))
    assert n > 0
    return out[:n].tobytes()


def encode_split(bands_flat, w, h, levels, lc, nthreads):
    """encode() through the band-parallel split (encoder.cpp tree_model_records
    + replay_events; nthreads <= 0: every band modelled, then replayed, serially)."""
    b = np.ascontiguousarray(bands_flat, np.int32)
    cap = w * h * 4 + 4096
    out = np.zeros(cap, np.uint8)
    s1, s2, s3 = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    n = lib().hc_encode_rec_split(b.ctypes.data, b.size, 1, w, h, levels, lc, out.ctypes.data, cap, nthreads,
                                  ctypes.byref(s1), ctypes.byref(s2), ctypes.byref(s3))
    assert n > 0
    return out[:n].tobytes()


def encode_compact(bands_flat, w, h, levels, lc):
    """encode() through the compacted-payload walk (encoder.cpp
    tree_encode_records_compact over the stream compact.hip writes)."""
    b = np.ascontiguousarray(bands_flat, np.int32)
    cap = w * h * 4 + 4096
    out = np.zeros(cap, np.uint8)
    n = lib().hc_encode_rec_compact(b.ctypes.data, b.size, 1, w, h, levels, lc, out.ctypes.data, cap)
    assert n > 0
    return out[:n].tobytes()


def decode(buf, w, h, levels, lc, total):
    """-> canonical band dump (int32) of one decoded plane (before TSUQi)."""
    b = np.frombuffer(buf, np.uint8).copy()
    out = np.zeros(total, np.int32)
    s = ctypes.c_double()
    lib().hc_decode(b.ctypes.data, len(buf), 1, w, h, levels, lc, out.ctypes.data, ctypes.byref(s))
    return out


def decode_compact(buf, w, h, levels, lc, total):
    """decode() with the finest level through tree_decode_compact, scattered
    back as k_dcmp_expand does."""
    b = np.frombuffer(buf, np.uint8).copy()
    out = np.zeros(total, np.int32)
    s = ctypes.c_double()
    lib().hc_decode_compact(b.ctypes.data, len(buf), 1, w, h, levels, lc, out.ctypes.data, ctypes.byref(s))
    return out
