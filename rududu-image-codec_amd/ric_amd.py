"""ric_amd -- Python mirror of the reference's src/lib codec interface over the
C-ABI in include/ric_gpu.h (librududu_amd.so).

Names follow the reference: ``Wavelet2D`` ~ CWavelet2D (src/lib/wavelet2d.h),
``MuxCodec`` ~ CMuxCodec (src/lib/muxcodec.h), ``Codec.compress`` /
``Codec.decompress`` ~ CompressImage / DecompressImage (src/ric/ric.cpp).

This module is plumbing for tests and the benchmark; the product is the HIP
library.  Loading fails loudly when the library is missing -- there is no CPU
fallback.  Device buffers are DeviceArray objects (HBM allocated by the
library's own HIP runtime, ric_device_alloc) or raw pointers; host buffers are
numpy arrays.
"""
import collections
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# RIC_AMD_LIB: another build of the library (A/B runs of a variant in one box call)
LIB_PATH = os.environ.get("RIC_AMD_LIB") or os.path.join(HERE, "librududu_amd.so")

RIC_OK, RIC_E_ARG, RIC_E_HIP, RIC_E_CAPACITY, RIC_E_FORMAT, RIC_E_STREAM = 0, -1, -2, -3, -4, -5
CDF97, CDF53, HAAR = 0, 1, 2

_P, _I, _S, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_float


class RicError(RuntimeError):
    def __init__(self, rc, what):
        self.rc = rc
        super().__init__("%s failed: status %d (%s)" % (what, rc, last_error()))


_lib = None


def lib():
    """Load librududu_amd.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("librududu_amd.so not built: run `python %s`" % os.path.join(HERE, "build.py"))
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "ric_version": (ctypes.c_char_p, []),
        "ric_device_count": (_I, []),
        "ric_last_error": (ctypes.c_char_p, []),
        "ric_wavelet_create": (_I, [ctypes.POINTER(_P), _I, _I, _I, _I, _I]),
        "ric_wavelet_destroy": (None, [_P]),
        "ric_wavelet_set_stream": (_I, [_P, _P]),
        "ric_wavelet_set_host_threads": (_I, [_P, _I]),
        "ric_band_tsuq": (_I, [_P, _I, _I, ctypes.c_float, _P, _P, _P]),
        "ric_band_tsuqi": (_I, [_P, _I, _I]),
        "ric_band_sums": (_I, [_P, _I, _P, _P]),
        "ric_band_add": (_I, [_P, _I, _I]),
        "ric_band_clear": (_I, [_P, _I]),
        "ric_wavelet_sync": (_I, [_P]),
        "ric_set_weight": (_I, [_P, _I, _F]),
        "ric_transform": (_I, [_P, _P, _I, _I, _I]),
        "ric_transform_inv": (_I, [_P, _P, _I, _I, _I]),
        "ric_code_band": (_I, [_P, _P, _I, _I]),
        "ric_quantize": (_I, [_P, _I, _I]),
        "ric_transform_quantize": (_I, [_P, _P, _I, _I, _I, _I, _I]),
        "ric_decode_band": (_I, [_P, _P]),
        "ric_tsuqi": (_I, [_P, _I]),
        "ric_tsuq": (_I, [_P, _I, _F, ctypes.POINTER(ctypes.c_uint)]),
        "ric_band_count": (_I, [_P]),
        "ric_band_info": (_I, [_P, _I, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_F)]),
        "ric_band_read": (_I, [_P, _I, _P]),
        "ric_band_write": (_I, [_P, _I, _P]),
        "ric_band_host": (_I, [_P, _I, ctypes.POINTER(_P), ctypes.POINTER(_I)]),
        "ric_band_host_ref": (_I, [_P, _I, ctypes.POINTER(_P), ctypes.POINTER(_I)]),
        "ric_mux_create_decoder_inplace": (_I, [ctypes.POINTER(_P), _P]),
        "ric_mux_reinit_encoder": (_I, [_P, _P, _S, ctypes.c_uint16]),
        "ric_mux_reinit_decoder": (_I, [_P, _P, _S]),
        "ric_mux_create_encoder": (_I, [ctypes.POINTER(_P), _P, _S, ctypes.c_uint16]),
        "ric_mux_create_decoder": (_I, [ctypes.POINTER(_P), _P, _S]),
        "ric_mux_end": (_I, [_P, ctypes.POINTER(_S)]),
        "ric_mux_size": (_S, [_P]),
        "ric_mux_destroy": (None, [_P]),
        "ric_codec_create": (_I, [ctypes.POINTER(_P), _I, _I, _I, _I]),
        "ric_codec_destroy": (None, [_P]),
        "ric_codec_set_stream": (_I, [_P, _P]),
        "ric_codec_set_host_threads": (_I, [_P, _I]),
        "ric_video_set_host_threads": (_I, [_P, _I]),
        "ric_codec_encode": (_I, [_P, _P, _I, _I, _I, _P, _S, ctypes.POINTER(_S)]),
        "ric_codec_decode": (_I, [_P, _P, _S, _I, _P, _P, _I]),
        "ric_read_header": (_I, [_P, _S, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I),
                                 ctypes.POINTER(_I), ctypes.POINTER(_I)]),
        "ric_quants": (_I, [_I]),
        "ric_prof_enable": (_I, [_P, _I]),
        "ric_prof_read": (_I, [_P, _P, _P, _I]),
        "ric_codec_wavelet": (_P, [_P]),
        "ric_synth_image": (None, [_I, _I, _I, _I, _P]),
        "ric_diag_wgtrace": (_I, [_I, _P, _I]),
        "ric_diag_fault": (_I, [_I]),
        "ric_diag_deferred_frees": (ctypes.c_long, []),
        "ric_batch_create": (_I, [ctypes.POINTER(_P), _I, _I, _I, _I, _I, _I]),
        "ric_batch_destroy": (None, [_P]),
        "ric_batch_encode": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P]),
        "ric_batch_decode": (_I, [_P, _P, _P, _I, _P, _I]),
        "ric_batch_roundtrip": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P]),
        "ric_batch_prof_enable": (_I, [_P, _I]),
        "ric_batch_encode_gpu": (_I, [_P, _P, _I, _I, _I, _P, ctypes.c_size_t, ctypes.c_size_t, _P]),
        "ric_batch_set_digests": (_I, [_P, _P, ctypes.c_long]),
        "ric_batch_hybrid_config": (_I, [_P, _I, ctypes.c_size_t]),
        "ric_batch_hybrid_config_ex": (_I, [_P, _I, ctypes.c_size_t, ctypes.c_long]),
        "ric_batch_hybrid_times": (_I, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
        "ric_batch_hybrid_fallbacks": (_I, [_P, ctypes.POINTER(ctypes.c_int)]),
        "ric_batch_decode_gpu": (_I, [_P, _P, ctypes.c_size_t, _P, _I, _P]),
        "ric_diag_gdec_dbg": (_I, [_P]),
        "ric_batch_roundtrip_hybrid": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
        "ric_batch_diag_gpu": (_I, [_P, _P, _I, _I, _I, _I, _P]),
        "ric_batch_diag_gpu_encode": (_I, [_P, _P, _I, _I, _I, _I]),
        "ric_batch_prof_read": (_I, [_P, _P, _P, _P, _I]),
        "ric_video_create": (_I, [ctypes.POINTER(_P), _I, _I, _I, _I, _I]),
        "ric_video_destroy": (None, [_P]),
        "ric_video_set_quant": (_I, [_P, _I]),
        "ric_video_encode": (_I, [_P, _P, _I, _I, _P, _S, ctypes.POINTER(_I)]),
        "ric_video_decode": (_I, [_P, _P, _S, ctypes.POINTER(_I)]),
        "ric_video_output": (_I, [_P, _P, _I, _I]),
        "ric_video_motion": (_I, [_P, _P]),
        "ric_device_alloc": (_I, [_I, _S, ctypes.POINTER(_P)]),
        "ric_device_free": (_I, [_P]),
        "ric_host_alloc": (_I, [_S, ctypes.POINTER(_P)]),
        "ric_host_free": (_I, [_P]),
        "ric_device_copy": (_I, [_I, _P, _P, _S, _I]),
        "ric_device_memset": (_I, [_I, _P, _I, _S]),
        "ric_device_sync": (_I, [_I]),
        "ric_device_digests": (_I, [_I, _P, _I, _P, _P, _P]),
        "ric_host_digests": (_I, [_P, _I, _P, _P, _P]),
        "ric_device_pack_h2d": (_I, [_I, _P, _I, _P, _P, _P, _P]),
        "ric_comm_unique_id": (_I, [_P, _S]),
        "ric_comm_create": (_I, [ctypes.POINTER(_P), _P, _I, _I, _I]),
        "ric_comm_destroy": (None, [_P]),
        "ric_comm_allreduce_f64": (_I, [_P, _P, _I, _I]),
        "ric_comm_sendrecv": (_I, [_P, _I, _P, _P, _P, _P]),
        "ric_batch_set_ready": (_I, [_P, _P, ctypes.c_long]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    _lib = L
    return L


def exported_symbols():
    """Names of the C-ABI entry points this binding expects."""
    lib()
    return [n for n in dir(_lib) if n.startswith("ric_")]


def last_error():
    return lib().ric_last_error().decode(errors="replace")


def _chk(rc, what):
    if rc != RIC_OK:
        raise RicError(rc, what)


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    raise TypeError(type(x))


def quants(idx):
    return lib().ric_quants(idx)


PROF_STAGES = ["fwd_l0", "fwd", "quant", "d2h", "host_enc", "host_dec", "h2d", "dequant", "inv",
               "pix_in", "pix_out"]


def synth(w, h, channels=1, frame=0):
    """SURVEY.md §8(d) synthetic image (channels, h, w) uint8, generated by the library."""
    out = np.empty((channels, h, w), np.uint8)
    lib().ric_synth_image(w, h, channels, frame, out.ctypes.data)
    return out


RIC_COPY_H2D, RIC_COPY_D2H, RIC_COPY_D2D = 1, 2, 3
RIC_RED_SUM, RIC_RED_MAX, RIC_RED_MIN = 0, 1, 2


class DeviceArray:
    """An HBM buffer allocated by the library's own HIP runtime
    (ric_device_alloc), with a shape and a numpy dtype.  data_ptr() is what the
    C-ABI takes; numpy() reads it back.  The plumbing for callers with no HIP
    runtime of their own: only the library's runtime is ever mapped."""

    def __init__(self, shape, dtype=np.uint8, device=0, zero=False):
        self.shape = tuple(int(s) for s in shape) if hasattr(shape, "__len__") else (int(shape),)
        self.dtype = np.dtype(dtype)
        self.device = device
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        p = _P()
        _chk(lib().ric_device_alloc(device, self.nbytes, ctypes.byref(p)), "ric_device_alloc(%d bytes)" % self.nbytes)
        self._p = p.value
        if zero:
            self.zero()

    @classmethod
    def from_numpy(cls, a, device=0):
        a = np.ascontiguousarray(a)
        d = cls(a.shape, a.dtype, device)
        d.copy_from(a)
        return d

    def empty_like(self):
        return DeviceArray(self.shape, self.dtype, self.device)

    def zeros_like(self):
        return DeviceArray(self.shape, self.dtype, self.device, zero=True)

    def data_ptr(self):
        return self._p

    def copy_from(self, a):
        a = np.ascontiguousarray(a, self.dtype)
        if a.nbytes != self.nbytes:
            raise ValueError("size mismatch: %d vs %d bytes" % (a.nbytes, self.nbytes))
        _chk(lib().ric_device_copy(self.device, self._p, a.ctypes.data, self.nbytes, RIC_COPY_H2D), "H2D copy")

    def numpy(self):
        out = np.empty(self.shape, self.dtype)
        _chk(lib().ric_device_copy(self.device, out.ctypes.data, self._p, self.nbytes, RIC_COPY_D2H), "D2H copy")
        return out

    def zero(self):
        _chk(lib().ric_device_memset(self.device, self._p, 0, self.nbytes), "memset")

    def __del__(self):
        p = getattr(self, "_p", None)
        if p and _lib is not None:
            _lib.ric_device_free(p)
            self._p = None


class _Pinned:
    def __init__(self, n):
        p = _P()
        _chk(lib().ric_host_alloc(n, ctypes.byref(p)), "ric_host_alloc")
        self.p = p.value

    def __del__(self):
        if getattr(self, "p", None) and _lib is not None:
            _lib.ric_host_free(self.p)
            self.p = None


def pinned_array(n):
    """A uint8 numpy array of n bytes in pinned host memory (ric_host_alloc),
    freed with the array."""
    holder = _Pinned(n)
    buf = (ctypes.c_uint8 * n).from_address(holder.p)
    a = np.frombuffer(buf, np.uint8)
    a_base = a.base                    # the ctypes buffer; keep the holder alive with it
    a_base._holder = holder
    return a


def device_sync(device=0):
    _chk(lib().ric_device_sync(device), "ric_device_sync")


def device_digests(device, base, offs, lens):
    """ric_device_digests: the 64-bit digest (ric_batch_set_digests' formula) of
    each device byte run base + offs[i], lens[i] bytes."""
    n = len(offs)
    o = np.ascontiguousarray(offs, np.uint64)
    ln = np.ascontiguousarray(lens, np.uint64)
    out = np.zeros(n, np.uint64)
    if n:
        _chk(lib().ric_device_digests(device, _ptr(base), n, o.ctypes.data, ln.ctypes.data, out.ctypes.data),
             "ric_device_digests")
    return out


def host_digests(base, offs, lens):
    """ric_host_digests: the same digest over host byte runs of `base` (a numpy
    array or a pointer)."""
    n = len(offs)
    o = np.ascontiguousarray(offs, np.uint64)
    ln = np.ascontiguousarray(lens, np.uint64)
    out = np.zeros(n, np.uint64)
    if n:
        _chk(lib().ric_host_digests(_ptr(base), n, o.ctypes.data, ln.ctypes.data, out.ctypes.data), "ric_host_digests")
    return out


def device_pack_h2d(device, dst, srcs, offs):
    """ric_device_pack_h2d: host byte runs srcs[i] (numpy uint8 arrays or bytes)
    packed at device dst + offs[i] in one copy; returns their digests."""
    n = len(srcs)
    arrs = [np.frombuffer(x, np.uint8) if not isinstance(x, np.ndarray) else np.ascontiguousarray(x).reshape(-1)
            for x in srcs]
    ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
    ln = np.ascontiguousarray([a.size for a in arrs], np.uint64)
    o = np.ascontiguousarray(offs, np.uint64)
    dig = np.zeros(n, np.uint64)
    if n:
        _chk(lib().ric_device_pack_h2d(device, _ptr(dst), n, ptrs, ln.ctypes.data, o.ctypes.data, dig.ctypes.data),
             "ric_device_pack_h2d")
    return dig


class Comm:
    """ric_comm: one RCCL communicator of this process (one process per GPU)."""
    ID_BYTES = 128

    @staticmethod
    def unique_id():
        b = np.zeros(Comm.ID_BYTES, np.uint8)
        _chk(lib().ric_comm_unique_id(b.ctypes.data, b.size), "ric_comm_unique_id")
        return b.tobytes()

    def __init__(self, uid, nranks, rank, device=0):
        b = np.frombuffer(uid, np.uint8).copy()
        h = _P()
        _chk(lib().ric_comm_create(ctypes.byref(h), b.ctypes.data, nranks, rank, device), "ric_comm_create")
        self.h, self.nranks, self.rank, self.device = h, nranks, rank, device

    def allreduce(self, vals, op=RIC_RED_SUM):
        v = np.ascontiguousarray(vals, np.float64).copy()
        _chk(lib().ric_comm_allreduce_f64(self.h, v.ctypes.data, v.size, op), "ric_comm_allreduce_f64")
        return v

    def sendrecv(self, ops):
        """ops: [(peer, is_send, device buffer or pointer, nbytes)] as one group."""
        n = len(ops)
        peer = (ctypes.c_int * n)(*[o[0] for o in ops])
        snd = (ctypes.c_int * n)(*[int(bool(o[1])) for o in ops])
        bufs = (ctypes.c_void_p * n)(*[_ptr(o[2]) for o in ops])
        nb = (ctypes.c_size_t * n)(*[int(o[3]) for o in ops])
        _chk(lib().ric_comm_sendrecv(self.h, n, peer, snd, bufs, nb), "ric_comm_sendrecv")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ric_comm_destroy(self.h)
            self.h = None


def _prof_enable(handle, on):
    _chk(lib().ric_prof_enable(handle, int(on)), "prof_enable")


def _prof_read(handle):
    ms = np.zeros(len(PROF_STAGES), np.float64)
    n = np.zeros(len(PROF_STAGES), np.int64)
    lib().ric_prof_read(handle, ms.ctypes.data, n.ctypes.data, len(PROF_STAGES))
    return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(PROF_STAGES)}


class MuxCodec:
    """CMuxCodec: host serial range coder / raw-bit multiplexer."""

    def __init__(self, buf, first_word=None, length=None):
        self._buf = buf
        h = _P()
        if first_word is not None:       # encoder: CMuxCodec(pStream, firstWord); buf None: CMuxCodec(0, 0)
            _chk(lib().ric_mux_create_encoder(ctypes.byref(h), _ptr(buf), buf.nbytes if buf is not None else 0,
                                              first_word), "CMuxCodec(enc)")
            self.encoder = True
        else:                            # decoder: CMuxCodec(pStream)
            n = buf.nbytes if length is None else length
            _chk(lib().ric_mux_create_decoder(ctypes.byref(h), _ptr(buf), n), "CMuxCodec(dec)")
            self.encoder = False
        self.h = h

    def initCoder(self, first_word, buf):
        """CMuxCodec::initCoder (src/lib/muxcodec.h:104); buf None keeps the output position."""
        if buf is not None:
            self._buf = buf
        _chk(lib().ric_mux_reinit_encoder(self.h, _ptr(buf), buf.nbytes if buf is not None else 0, first_word),
             "initCoder")
        self.encoder = True

    def initDecoder(self, buf, length=None):
        """CMuxCodec::initDecoder (src/lib/muxcodec.h:105), bounded to `length` bytes of buf (all of it by default)."""
        if buf is not None:
            self._buf = buf
        n = 0 if buf is None else (buf.nbytes if length is None else length)
        _chk(lib().ric_mux_reinit_decoder(self.h, _ptr(buf), n), "initDecoder")
        self.encoder = False

    def endCoding(self):
        n = _S()
        _chk(lib().ric_mux_end(self.h, ctypes.byref(n)), "endCoding")
        return n.value

    def getSize(self):
        return lib().ric_mux_size(self.h)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ric_mux_destroy(self.h)
            self.h = None


class Wavelet2D:
    """CWavelet2D(x, y, level, level_chg): band pyramid resident in HBM."""

    def __init__(self, x, y, level, level_chg=0, device=0):
        h = _P()
        _chk(lib().ric_wavelet_create(ctypes.byref(h), x, y, level, level_chg, device), "CWavelet2D")
        self.h = h
        self.DimX, self.DimY = x, y

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ric_wavelet_destroy(self.h)
            self.h = None

    def set_stream(self, stream_ptr):
        _chk(lib().ric_wavelet_set_stream(self.h, stream_ptr), "set_stream")

    def set_host_threads(self, n):
        """CodeBand's serial half over n host threads (bands modelled in parallel)."""
        _chk(lib().ric_wavelet_set_host_threads(self.h, n), "set_host_threads")

    # CBand's operations on band i (device): TSUQ, TSUQi, Mean's sums, Add, Clear
    def band_tsuq(self, i, quant, thres):
        """-> (count, max, min)"""
        c, mx, mn = ctypes.c_uint(), ctypes.c_int(), ctypes.c_int()
        _chk(lib().ric_band_tsuq(self.h, i, quant, thres, ctypes.byref(c), ctypes.byref(mx), ctypes.byref(mn)),
             "CBand::TSUQ")
        return c.value, mx.value, mn.value

    def band_tsuqi(self, i, quant):
        _chk(lib().ric_band_tsuqi(self.h, i, quant), "CBand::TSUQi")

    def band_sums(self, i):
        s, ss = ctypes.c_int64(), ctypes.c_int64()
        _chk(lib().ric_band_sums(self.h, i, ctypes.byref(s), ctypes.byref(ss)), "CBand::Mean")
        return s.value, ss.value

    def band_add(self, i, val):
        _chk(lib().ric_band_add(self.h, i, val), "CBand::Add")

    def band_clear(self, i):
        _chk(lib().ric_band_clear(self.h, i), "CBand::Clear")

    def sync(self):
        _chk(lib().ric_wavelet_sync(self.h), "sync")

    def SetWeight(self, t, baseWeight=1.0):
        _chk(lib().ric_set_weight(self.h, t, baseWeight), "SetWeight")

    def Transform(self, image, stride, t, on_device=None):
        dev = on_device if on_device is not None else not isinstance(image, np.ndarray)
        _chk(lib().ric_transform(self.h, _ptr(image), stride, t, int(dev)), "Transform")

    def TransformI(self, image, stride, t, on_device=None):
        dev = on_device if on_device is not None else not isinstance(image, np.ndarray)
        _chk(lib().ric_transform_inv(self.h, _ptr(image), stride, t, int(dev)), "TransformI")

    def CodeBand(self, codec, quant, lam):
        _chk(lib().ric_code_band(self.h, codec.h, quant, lam), "CodeBand")

    def Quantize(self, quant, lam):
        """Device half of CodeBand only (buildTree + LL TSUQ + block records)."""
        _chk(lib().ric_quantize(self.h, quant, lam), "Quantize")

    def TransformQuantize(self, image, stride, t, quant, lam, on_device=None):
        """Transform + device half of CodeBand as one fused pass (synchronous)."""
        dev = on_device if on_device is not None else not isinstance(image, np.ndarray)
        _chk(lib().ric_transform_quantize(self.h, _ptr(image), stride, t, int(dev), quant, lam),
             "TransformQuantize")

    def DecodeBand(self, codec):
        rc = lib().ric_decode_band(self.h, codec.h)
        if rc not in (RIC_OK, RIC_E_STREAM):
            _chk(rc, "DecodeBand")
        return rc

    def TSUQi(self, quant):
        _chk(lib().ric_tsuqi(self.h, quant), "TSUQi")

    def TSUQ(self, quant, thres):
        n = ctypes.c_uint()
        _chk(lib().ric_tsuq(self.h, quant, thres, ctypes.byref(n)), "TSUQ")
        return n.value

    def band_count(self):
        return lib().ric_band_count(self.h)

    def band_info(self, i):
        dx, dy, isint, w = _I(), _I(), _I(), _F()
        _chk(lib().ric_band_info(self.h, i, ctypes.byref(dx), ctypes.byref(dy), ctypes.byref(isint),
                                 ctypes.byref(w)), "band_info")
        return dx.value, dy.value, isint.value, w.value

    def bands(self):
        """All bands in canonical order (finest->coarsest D,H,V; then LL)."""
        out = []
        for i in range(self.band_count()):
            dx, dy, _, _ = self.band_info(i)
            a = np.zeros((dy, dx), np.int32)
            _chk(lib().ric_band_read(self.h, i, a.ctypes.data), "band_read")
            out.append(a)
        return out

    def prof_enable(self, on=True):
        _prof_enable(self.h, on)

    def prof_read(self):
        return _prof_read(self.h)

    def write_band(self, i, arr):
        a = np.ascontiguousarray(arr, np.int32)
        _chk(lib().ric_band_write(self.h, i, a.ctypes.data), "band_write")


BATCH_STAGES = (["pix_in"] + ["fwd_l%d" % l for l in range(8)] + ["d2h", "host_enc", "host_dec", "h2d"] +
                ["inv_l%d" % l for l in range(8)] + ["pix_out", "gpu_enc", "gpu_dec", "d2h_values", "gpu_rt", "dcmp_expand", "compact"])


_PTRS_CACHE = collections.OrderedDict()


def _ptrs(xs):
    """A ctypes array of the buffers' addresses.  Long lists (a serving step's
    ~4000 frames, outputs and stream buffers, the same objects every step) are
    kept in a small LRU cache keyed by the objects' identities; the entry holds
    the objects, so an identity cannot be reused while it is cached.  Building
    the three arrays took ~10 ms per step, with the GPU idle between calls."""
    n = len(xs)
    key = None
    if n >= 256:
        key = tuple(map(id, xs))
        hit = _PTRS_CACHE.get(key)
        if hit is not None:
            _PTRS_CACHE.move_to_end(key)
            return hit[1]
        # a prefix of a cached list (the step's frame count moves with the
        # host/GPU balance): a view of the cached array's first n entries
        for k, (objs, arr) in _PTRS_CACHE.items():
            if len(k) > n and k[:n] == key:
                return (ctypes.c_void_p * n).from_buffer(arr)
    a = (ctypes.c_void_p * n)()
    for i, x in enumerate(xs):
        a[i] = _ptr(x)
    if key is not None:
        _PTRS_CACHE[key] = (list(xs), a)
        while len(_PTRS_CACHE) > 8:
            _PTRS_CACHE.popitem(last=False)
    return a


class Batch:
    """ric_batch: CompressImage / DecompressImage over groups of up to `slots`
    frames (one GPU launch per level per group, a native pool of `threads`
    host coder threads).  Frames are (channels, h, w) uint8 numpy arrays or
    device tensors / pointers."""

    def __init__(self, w, h, channels=1, slots=16, threads=16, device=0):
        hd = _P()
        _chk(lib().ric_batch_create(ctypes.byref(hd), w, h, channels, slots, threads, device), "ric_batch_create")
        self.h = hd
        self.w, self.hgt, self.channels, self.slots = w, h, channels, slots
        self.cap = w * h * channels * 2 + 65536
        self._outs = []

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ric_batch_destroy(self.h)
            self.h = None

    def _out_bufs(self, n):
        while len(self._outs) < n:
            self._outs.append(np.empty(self.cap, np.uint8))
        return self._outs[:n]

    def compress(self, frames, q=9, trans=None, on_device=None):
        """Returns the list of .ric files (bytes)."""
        if trans is None:
            trans = CDF53 if q == 0 else CDF97
        n = len(frames)
        dev = on_device if on_device is not None else not isinstance(frames[0], np.ndarray)
        if not dev:
            frames = [np.ascontiguousarray(f, np.uint8) for f in frames]
        outs = self._out_bufs(n)
        caps = (ctypes.c_size_t * n)(*([self.cap] * n))
        lens = (ctypes.c_size_t * n)()
        _chk(lib().ric_batch_encode(self.h, _ptrs(frames), n, int(dev), q, trans, _ptrs(outs), caps, lens),
             "ric_batch_encode")
        return [outs[i][:lens[i]].tobytes() for i in range(n)]

    def compress_gpu(self, frames, out, ostride, q=9, trans=0):
        """Whole encode on the GPU (ric_batch_encode_gpu): frames are device
        pixel pointers/tensors, out a device buffer of len(frames) * ostride
        bytes; returns the files' sizes (the files stay in device memory)."""
        n = len(frames)
        lens = (ctypes.c_size_t * n)()
        _chk(lib().ric_batch_encode_gpu(self.h, _ptrs(frames), n, q, trans, _ptr(out), ostride, ostride, lens),
             "ric_batch_encode_gpu")
        return [lens[i] for i in range(n)]

    def decompress_gpu(self, src, istride, lens, pix_out):
        """Whole decode on the GPU (ric_batch_decode_gpu): src a device buffer
        holding the files at multiples of istride, pix_out device tensors."""
        n = len(lens)
        ls = (ctypes.c_size_t * n)(*lens)
        rc = lib().ric_batch_decode_gpu(self.h, _ptr(src), istride, ls, n, _ptrs(pix_out))
        if rc not in (RIC_OK, RIC_E_STREAM):
            _chk(rc, "ric_batch_decode_gpu")
        return rc

    def decompress(self, rics, pix_out=None):
        """Host mode: returns a list of (channels, h, w) uint8 arrays.  Device
        mode: pass device tensors / pointers in pix_out.  Returns the status
        (RIC_OK or RIC_E_STREAM) in device mode."""
        n = len(rics)
        bufs = [np.frombuffer(r, np.uint8) for r in rics]
        lens = (ctypes.c_size_t * n)(*[len(r) for r in rics])
        if pix_out is None:
            outs = [np.zeros((self.channels, self.hgt, self.w), np.uint8) for _ in range(n)]
            rc = lib().ric_batch_decode(self.h, _ptrs(bufs), lens, n, _ptrs(outs), 0)
            if rc not in (RIC_OK, RIC_E_STREAM):
                _chk(rc, "ric_batch_decode")
            return outs
        rc = lib().ric_batch_decode(self.h, _ptrs(bufs), lens, n, _ptrs(pix_out), 1)
        if rc not in (RIC_OK, RIC_E_STREAM):
            _chk(rc, "ric_batch_decode")
        return rc

    def roundtrip(self, frames, pix_out, q=9, trans=0, allow_stream_err=False):
        """Encode then decode every frame (device pixels in and out), groups
        pipelined; returns the .ric files' sizes and keeps the files in
        self.streams(n).  RIC_E_STREAM (a decoder ran past its stream: only
        the reference's own desynchronising geometries do that)
        raises unless allow_stream_err."""
        n = len(frames)
        outs = self._out_bufs(n)
        caps = (ctypes.c_size_t * n)(*([self.cap] * n))
        lens = (ctypes.c_size_t * n)()
        self._streams = None
        rc = lib().ric_batch_roundtrip(self.h, _ptrs(frames), n, q, trans, _ptrs(outs), caps, lens, _ptrs(pix_out))
        if rc != RIC_OK and not (allow_stream_err and rc == RIC_E_STREAM):
            _chk(rc, "ric_batch_roundtrip")
        self._lens = [lens[i] for i in range(n)]
        return self._lens

    def set_digests(self, dev_digests, n):
        """Per frame of the next calls, the 64-bit digest of its decoded pixels
        into dev_digests[i] (a device uint64 DeviceArray / pointer; n = 0: off).
        The buffer is kept referenced here while the library holds its pointer."""
        _chk(lib().ric_batch_set_digests(self.h, _ptr(dev_digests) if n else None, n), "ric_batch_set_digests")
        self._digests = dev_digests if n else None

    def set_ready(self, words, n):
        """ric_batch_set_ready: words (a uint32 numpy array) gets frame i's
        .ric length as soon as its file is complete (n = 0: off); kept
        referenced here while the library holds its pointer."""
        if n and (not isinstance(words, np.ndarray) or words.dtype != np.uint32 or words.size < n):
            raise ValueError("set_ready: a uint32 numpy array of at least n words")
        _chk(lib().ric_batch_set_ready(self.h, words.ctypes.data if n else None, n), "ric_batch_set_ready")
        self._ready = words if n else None

    def hybrid_config(self, pool_frames, stream_cap, value_cap=-1):
        """Pool of the GPU stream coder (ric_batch_hybrid_config_ex): value_cap
        the finest bands' compacted capacity per plane (-1 the default, 0 dense)."""
        _chk(lib().ric_batch_hybrid_config_ex(self.h, pool_frames, stream_cap, value_cap), "ric_batch_hybrid_config_ex")

    def hybrid_times(self):
        """(host side, GPU side) end of the last roundtrip_hybrid, ms from its start."""
        hm, gm = ctypes.c_double(), ctypes.c_double()
        _chk(lib().ric_batch_hybrid_times(self.h, ctypes.byref(hm), ctypes.byref(gm)), "ric_batch_hybrid_times")
        return hm.value, gm.value

    def hybrid_fallbacks(self):
        """Frames of the last roundtrip_hybrid over the pool's value capacity
        (round-tripped on the host instead)."""
        n = ctypes.c_int(0)
        _chk(lib().ric_batch_hybrid_fallbacks(self.h, ctypes.byref(n)), "ric_batch_hybrid_fallbacks")
        return n.value

    def roundtrip_hybrid(self, frames, pix_out, n_host, q=9, trans=0, gpu_decode=False, streams=None,
                         allow_stream_err=False):
        """ric_batch_roundtrip_hybrid: frames[:n_host] round trips on the host,
        the rest encoded by the GPU stream coder and decoded by the GPU stream
        decoder (gpu_decode 1), on the host (0), or per launch by whichever
        has room (2).  `streams`: one host buffer per frame (distinct: the
        library rejects aliased ones).  RIC_E_STREAM raises unless
        allow_stream_err."""
        n = len(frames)
        outs = streams if streams is not None else self._out_bufs(n)   # host buffers of the .ric files
        pf, po, pp = _ptrs(frames), _ptrs(outs), _ptrs(pix_out)
        caps = (ctypes.c_size_t * n)(*[o.size for o in outs])
        lens = (ctypes.c_size_t * n)()
        self._streams = outs
        rc = lib().ric_batch_roundtrip_hybrid(self.h, pf, n, n_host, int(gpu_decode), q, trans, po, caps, lens, pp)
        if rc != RIC_OK and not (allow_stream_err and rc == RIC_E_STREAM):
            _chk(rc, "ric_batch_roundtrip_hybrid")
        self._lens = [lens[i] for i in range(n)]
        return self._lens

    def stream(self, i):
        bufs = getattr(self, "_streams", None) or self._outs
        return bufs[i][:self._lens[i]].tobytes()

    def diag_gpu(self, frames, q=9, trans=0, iters=1, pix_out=None):
        """GPU stages only (kernel timing), see ric_batch_diag_gpu."""
        po = _ptrs(pix_out) if pix_out is not None else None
        _chk(lib().ric_batch_diag_gpu(self.h, _ptrs(frames), len(frames), q, trans, iters, po), "ric_batch_diag_gpu")

    def diag_gpu_encode(self, frames, q=9, trans=0, iters=1):
        """The forward levels alone, back to back (ric_batch_diag_gpu_encode)."""
        _chk(lib().ric_batch_diag_gpu_encode(self.h, _ptrs(frames), len(frames), q, trans, iters),
             "ric_batch_diag_gpu_encode")

    def prof_enable(self, on=True):
        _chk(lib().ric_batch_prof_enable(self.h, int(on)), "ric_batch_prof_enable")

    def prof_read(self):
        k = len(BATCH_STAGES)
        ms = np.zeros(k, np.float64)
        fr = np.zeros(k, np.int64)
        ln = np.zeros(k, np.int64)
        lib().ric_batch_prof_read(self.h, ms.ctypes.data, fr.ctypes.data, ln.ctypes.data, k)
        return {s: (float(ms[i]), int(fr[i]), int(ln[i])) for i, s in enumerate(BATCH_STAGES)}


def read_header(ric):
    b = np.frombuffer(ric, np.uint8)
    w, h, c, q, t = _I(), _I(), _I(), _I(), _I()
    _chk(lib().ric_read_header(b.ctypes.data, len(ric), ctypes.byref(w), ctypes.byref(h), ctypes.byref(c),
                               ctypes.byref(q), ctypes.byref(t)), "read_header")
    return w.value, h.value, c.value, q.value, t.value


class Codec:
    """CompressImage / DecompressImage for one image geometry on one GPU."""

    def __init__(self, w, h, channels=1, device=0):
        hd = _P()
        _chk(lib().ric_codec_create(ctypes.byref(hd), w, h, channels, device), "ric_codec_create")
        self.h = hd
        self.w, self.hgt, self.channels = w, h, channels

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ric_codec_destroy(self.h)
            self.h = None

    def set_stream(self, stream_ptr):
        _chk(lib().ric_codec_set_stream(self.h, stream_ptr), "set_stream")

    def set_host_threads(self, n):
        """The encoder's serial stage over n host threads (bands modelled in
        parallel, one thread writing the stream): lower latency, same bytes."""
        _chk(lib().ric_codec_set_host_threads(self.h, n), "set_host_threads")

    def prof_enable(self, on=True):
        _prof_enable(lib().ric_codec_wavelet(self.h), on)

    def prof_read(self):
        return _prof_read(lib().ric_codec_wavelet(self.h))

    def compress(self, pix, q=9, trans=None, on_device=None):
        """pix: (channels, h, w) uint8 numpy array or device pointer/tensor.
        Returns the .ric file bytes."""
        if trans is None:
            trans = CDF53 if q == 0 else CDF97          # ric -t default (src/ric/ric.cpp:313)
        dev = on_device if on_device is not None else not isinstance(pix, np.ndarray)
        if not dev:
            pix = np.ascontiguousarray(pix, np.uint8)
        cap = self.w * self.hgt * self.channels * 2 + 65536
        out = getattr(self, "_out", None)          # reused: no fresh pages per frame
        if out is None or out.size < cap:
            out = self._out = np.empty(cap, np.uint8)
        n = _S()
        _chk(lib().ric_codec_encode(self.h, _ptr(pix), int(dev), q, trans, out.ctypes.data, cap, ctypes.byref(n)),
             "CompressImage")
        return out[:n.value].tobytes()

    def decompress(self, ric, dither=False, pix_out=None, planes_out=None):
        """Host mode (default): returns (pix uint8 (c,h,w), planes int16 (c,h,w)).
        Device mode: pass device pointers/tensors in pix_out / planes_out."""
        b = np.frombuffer(ric, np.uint8)
        if pix_out is None and planes_out is None:
            pix = np.zeros((self.channels, self.hgt, self.w), np.uint8)
            planes = np.zeros((self.channels, self.hgt, self.w), np.int16)
            rc = lib().ric_codec_decode(self.h, b.ctypes.data, len(ric), int(dither), pix.ctypes.data,
                                        planes.ctypes.data, 0)
            if rc not in (RIC_OK, RIC_E_STREAM):
                _chk(rc, "DecompressImage")
            return pix, planes
        rc = lib().ric_codec_decode(self.h, b.ctypes.data, len(ric), int(dither), _ptr(pix_out),
                                    _ptr(planes_out), 1)
        if rc not in (RIC_OK, RIC_E_STREAM):
            _chk(rc, "DecompressImage")
        return rc


class VideoCodec:
    """CRududuCodec (src/lib/rududucodec.{h,cpp}): the reference's video codec
    on the GPU.  encoder=True is CRududuCodec(encode, ...), else decode.
    Frames are (3, h, w) uint8 arrays of planes R, G, B with the bottom row
    first (CImage::inputSGI), host numpy or device tensors."""

    def __init__(self, encoder, w, h, component=3, device=0):
        hd = _P()
        _chk(lib().ric_video_create(ctypes.byref(hd), int(bool(encoder)), w, h, component, device), "CRududuCodec")
        self.h = hd
        self.w, self.hgt = w, h
        self._quant = 0
        self._buf = np.zeros(w * h * 3 * 4 + 65536, np.uint8)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ric_video_destroy(self.h)
            self.h = None

    @property
    def quant(self):
        return self._quant

    @quant.setter
    def quant(self, q):
        _chk(lib().ric_video_set_quant(self.h, q), "CRududuCodec::quant")
        self._quant = q

    def set_host_threads(self, n):
        """the encoder's serial stage over n host threads (same bytes)"""
        _chk(lib().ric_video_set_host_threads(self.h, n), "set_host_threads")

    def encode(self, frame, stride=None, on_device=None):
        """CRududuCodec::encode: returns the frame's stream (size + 2 bytes)."""
        dev = on_device if on_device is not None else not isinstance(frame, np.ndarray)
        if not dev:
            frame = np.ascontiguousarray(frame, np.uint8)
        size = _I()
        _chk(lib().ric_video_encode(self.h, _ptr(frame), stride or self.w, int(dev), self._buf.ctypes.data,
                                    self._buf.nbytes, ctypes.byref(size)), "CRududuCodec::encode")
        return self._buf[:size.value + 2].tobytes()

    def decode(self, stream):
        """CRududuCodec::decode: returns getSize()."""
        b = np.frombuffer(stream, np.uint8)
        size = _I()
        rc = lib().ric_video_decode(self.h, b.ctypes.data, len(stream), ctypes.byref(size))
        if rc != RIC_OK:
            _chk(rc, "CRududuCodec::decode")
        return size.value

    def output(self, border=False):
        """*outImage of the last call: int16 planes Y, Co, Cg (3, h, w), or with
        the 15-sample border (3, h + 30, w + 30)."""
        b = 15 if border else 0
        out = np.zeros((3, self.hgt + 2 * b, self.w + 2 * b), np.int16)
        _chk(lib().ric_video_output(self.h, out.ctypes.data, int(bool(border)), 0), "outImage")
        return out

    def prediction(self):
        """diagnostics: the OBMC prediction image (predImage) with its border"""
        out = np.zeros((3, self.hgt + 30, self.w + 30), np.int16)
        _chk(lib().ric_video_output(self.h, out.ctypes.data, 2, 0), "predImage")
        return out

    def motion(self):
        """the motion field (h >> 3, w >> 3), uint32 (x low, y high; MV_INTRA 0x80008000)"""
        out = np.zeros((self.hgt >> 3, self.w >> 3), np.uint32)
        _chk(lib().ric_video_motion(self.h, out.ctypes.data), "motion field")
        return out
