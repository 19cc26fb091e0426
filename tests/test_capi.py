"""The C-ABI library: it loads, exports every entry point include/ric_gpu.h
declares, and its host-only helpers agree with the oracle.  Nothing here runs
a kernel (no GPU in this container); on a GPU-less host object creation must
fail loudly, never fall back to the CPU."""
import os
import re

import numpy as np
import pytest

import ric_amd
from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ric_gpu.h")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ric_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    names = declared()
    assert len(names) >= 30
    lib = ric_amd.lib()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    import inspect
    src = inspect.getsource(ric_amd)
    assert [n for n in declared() if n not in src] == []


def test_quants_and_header_helpers():
    for i in range(0, 60):
        assert ric_amd.quants(i) == O.quants(i)
    g = open(os.path.join(REPO, "tests", "golden", "rgb96x80_q5_t0_f7.ric"), "rb").read()
    assert ric_amd.read_header(g) == (96, 80, 3, 5, 0)
    with pytest.raises(ric_amd.RicError):
        ric_amd.read_header(b"RUD1" + g[4:])


@pytest.mark.parametrize("w,h,c,f", [(64, 48, 1, 0), (33, 47, 3, 5), (7680, 16, 1, 9)])
def test_synthetic_generator_matches_oracle(w, h, c, f):
    assert np.array_equal(ric_amd.synth(w, h, c, f), O.synth(w, h, c, f))


def test_no_gpu_fails_loudly():
    if ric_amd.lib().ric_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(ric_amd.RicError):
        ric_amd.Codec(64, 48, 1)
    with pytest.raises(ric_amd.RicError):
        ric_amd.Wavelet2D(64, 48, 5, 1)


def test_mux_capacity_is_explicit():
    # the encoder refuses to write past its buffer (the reference has no bound)
    buf = np.zeros(8, np.uint8)
    m = ric_amd.MuxCodec(buf, first_word=0)
    assert m.getSize() == 2
    assert m.endCoding() <= 8


def test_mux_reinit():
    """CMuxCodec(0, 0) + initCoder / initDecoder (src/lib/muxcodec.h:102-105,
    src/lib/rududucodec.cpp:36,89,123): one object, re-initialised per frame,
    serving as encoder and decoder."""
    m = ric_amd.MuxCodec(None, first_word=0)          # CMuxCodec(0, 0): no buffer yet
    with pytest.raises(ric_amd.RicError):
        m.endCoding()                                  # nothing to end into
    outs = []
    for k in range(3):
        buf = np.full(64, 0xAA, np.uint8)
        m.initCoder(0, buf)
        assert m.getSize() == 2                        # pStream - pInitStream after initCoder
        n = m.endCoding()
        assert n == 4 and m.getSize() == 2                # the 4 final bytes land in the ring slots buf[0..3]
        outs.append(buf[:n].tobytes())
    assert outs[0] == outs[1] == outs[2]               # the state is fully reset per frame
    m.initDecoder(np.frombuffer(outs[0], np.uint8).copy())
    assert not m.encoder and m.getSize() == 2
    m.initCoder(0, np.zeros(64, np.uint8))             # and back to an encoder
    assert m.encoder


def test_shim_compat_builds():
    """A caller in the reference's own call forms (CMuxCodec(pStream, 0),
    CMuxCodec(pStream), DBand/pLow members, (C*) pBand) compiles and links
    against include/rududu_gpu.hpp + librududu_amd.so (tests/native/shim_compat.cpp)."""
    import subprocess
    nat = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
    subprocess.run(["make", "-s", "-C", nat, "all"], check=True, capture_output=True, timeout=300)
    assert os.path.exists(os.path.join(nat, "shim_compat"))
